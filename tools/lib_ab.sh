# A/B of two builds of the library (dev tool): bash tools/lib_ab.sh libA.so libB.so
set -e
for L in "$@"; do
  echo "== $L"
  for cfg in "64 64 4096 1 1" "64 64 512 0 0"; do
    GPEMU_LIB=gp_emu_uqsa_amd/$L timeout -k 10 60 python tools/gemm_one.py $cfg 10
  done
  GPEMU_LIB=gp_emu_uqsa_amd/$L timeout -k 10 120 python tools/quick_time.py 16384 10 | grep phases
  GPEMU_LIB=gp_emu_uqsa_amd/$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-other-configs 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('bench', d['value'], d['extra']['single_eval_ms'])"
done
