# PMC passes (instruction fetch / issue stalls) of one layout, old vs new build.
set -o pipefail
mkdir -p gpurun_out/laypmc
export TMPDIR=/tmp
for v in head0 new; do
  DPOW_LIB_PATH=abt/$v.so timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/laypmc/${v}_a -o run -- python3 tools/layout_pmc.py 8 > gpurun_out/laypmc/${v}_a.out 2>&1 || exit 1
  DPOW_LIB_PATH=abt/$v.so timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/laypmc/${v}_b -o run -- python3 tools/layout_pmc.py 8 > gpurun_out/laypmc/${v}_b.out 2>&1 || exit 1
done
