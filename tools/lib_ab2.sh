# A/B of two library builds (dev tool): GEMM rates per layout, phase times, bench.
# usage: bash tools/lib_ab2.sh libA.so libB.so   (files under gp_emu_uqsa_amd/)
set -e
mkdir -p gpurun_out
for L in "$@"; do
  GPEMU_LIB=gp_emu_uqsa_amd/$L timeout -k 10 120 python3 tools/gemm_ab.py > gpurun_out/ab_gemm_$L.log 2>&1
  GPEMU_LIB=gp_emu_uqsa_amd/$L timeout -k 10 120 python3 tools/quick_time.py 16384 10 > gpurun_out/ab_qt_$L.log 2>&1
done
for L in "$@"; do
  GPEMU_LIB=gp_emu_uqsa_amd/$L timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-other-configs > gpurun_out/ab_bench_$L.json 2>/dev/null
done
for L in "$@"; do
  echo "== $L"; cat gpurun_out/ab_gemm_$L.log; grep phases gpurun_out/ab_qt_$L.log
  python3 -c "import json;d=json.loads(open('gpurun_out/ab_bench_$L.json').read().strip().splitlines()[-1]);print('bench',round(d['value'],3),'single',round(d['extra']['single_eval_ms'],2))"
done
