bash tools/gpu_driver_check.sh r02h_driver && bash tools/profile_gpu.sh r02h pmc > gpurun_out/r02h_prof.out 2>&1
