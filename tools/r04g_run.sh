# round-4 check (dev tool): padded diagonal-block layout (micro, chain trace, phases) and
# the row-block objective's kernel breakdown at P = 1 (loopback)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_micro.sh > gpurun_out/micro_r04g.log 2>&1 || exit 1
P=gp_emu_uqsa_amd/libgpemu_pad.so
for n in 16384 4096; do GPEMU_LIB=$P timeout -k 10 120 python3 tools/quick_time.py $n 10 || exit 1; done > gpurun_out/qt_r04g_pad.log 2>&1
for n in 16384 4096; do GPEMU_LIB=gp_emu_uqsa_amd/libgpemu_pad_trace.so timeout -k 10 120 python3 tools/chol_trace.py $n || exit 1; done > gpurun_out/chol_trace_r04g_pad.log 2>&1
GPEMU_LIB=$P timeout -k 10 120 python3 tools/small_n_time.py > gpurun_out/small_n_r04g_pad.log 2>&1 || exit 1
timeout -k 10 240 python3 tools/dist_objective.py --loopback 1 --points 16384 --dims 10 > gpurun_out/dist_value_r04g.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_dist_r04g -o dist -- python3 tools/dist_objective.py --loopback 1 --points 16384 --dims 10 --grad --reps 2 > gpurun_out/dist_prof_r04g.log 2>&1
