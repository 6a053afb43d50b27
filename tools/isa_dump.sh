#!/bin/bash
# Device-only disassembly of every kernel translation unit of libdpow.so (the 8 (NBLK, SH) units,
# the 2 chunk-length-spanning units, search_ctrl.hip), one .s per unit, into DIR: a refactor of
# the kernel sources that claims to change nothing is checked by diffing two dumps.
#   bash tools/isa_dump.sh DIR [extra hipcc flags]
set -e
out=${1:?dir}; shift
mkdir -p "$out"
cd "$(dirname "$0")/../distributed-proof-of-work_amd/csrc"
L=/opt/rocm/lib/llvm/bin
F="-O3 -std=c++17 -DDPOW_NC=2 --offload-arch=gfx950 -munsafe-fp-atomics --cuda-device-only -c"
unit() {  # name src flags...
    local name=$1 src=$2; shift 2
    /opt/rocm/bin/hipcc $F "$@" "$src" -o "$out/$name.o"
    $L/clang-offload-bundler --type=o --input="$out/$name.o" --unbundle \
        --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output="$out/$name.co"
    $L/llvm-objdump -d --no-show-raw-insn "$out/$name.co" | sed 1,3d > "$out/$name.s"
    rm -f "$out/$name.o" "$out/$name.co"
}
for v in 1_0 1_1 1_2 1_3 2_0 2_1 2_2 2_3; do
    unit v$v md5_variant.hip -DDPOW_VNBLK=${v%_*} -DDPOW_VSH=${v#*_} "$@" &
done
unit ls1_0 md5_variant.hip -DDPOW_VLS=1 -DDPOW_VNBLK=1 -DDPOW_VSH=0 "$@" &
unit ls2_0 md5_variant.hip -DDPOW_VLS=1 -DDPOW_VNBLK=2 -DDPOW_VSH=0 "$@" &
unit ctrl search_ctrl.hip "$@" &
wait
