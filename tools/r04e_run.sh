# round-4 check (dev tool): swizzle micro-check, the -m gpu suite + timings of the head,
# then the swizzled-LDS and no-split-K builds' timings
mkdir -p gpurun_out
bash tools/gpu_micro.sh > gpurun_out/micro_r04e.log 2>&1 || exit 1
bash tools/gpu_check.sh r04e || exit 1
X=gp_emu_uqsa_amd/libgpemu_xor.so
GPEMU_LIB=$X timeout -k 10 300 python -u -m pytest tests/test_gpu_objective.py -x -q --timeout 120 --timeout-method thread > gpurun_out/xor_tests_r04e.log 2>&1 || exit 1
for n in 16384 4096; do GPEMU_LIB=$X timeout -k 10 120 python3 tools/quick_time.py $n 10 || exit 1; done > gpurun_out/qt_r04e_xor.log 2>&1
GPEMU_LIB=$X timeout -k 10 120 python3 tools/small_n_time.py > gpurun_out/small_n_r04e_xor.log 2>&1 || exit 1
N=gp_emu_uqsa_amd/libgpemu_nosk.so
GPEMU_LIB=$N timeout -k 10 120 python3 tools/small_n_time.py > gpurun_out/small_n_r04e_nosk.log 2>&1 || exit 1
GPEMU_LIB=$N timeout -k 10 120 python3 tools/quick_time.py 4096 10 > gpurun_out/qt_r04e_nosk.log 2>&1
Q=gp_emu_uqsa_amd/libgpemu_pipe.so
GPEMU_LIB=$Q timeout -k 10 300 python -u -m pytest tests/test_gpu_objective.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pipe_tests_r04e.log 2>&1 || exit 1
for n in 16384 4096; do GPEMU_LIB=$Q timeout -k 10 120 python3 tools/quick_time.py $n 10 || exit 1; done > gpurun_out/qt_r04e_pipe.log 2>&1
GPEMU_LIB=$Q timeout -k 10 120 python3 tools/small_n_time.py > gpurun_out/small_n_r04e_pipe.log 2>&1
