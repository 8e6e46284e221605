set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do for k in 2 3; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-other-configs --steps 12 --concurrent $k > gpurun_out/conc_$k.json 2>/dev/null || exit 1
  python3 -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('k', sys.argv[2], round(r['value'], 3), round(r['ms_per_step'], 2))" gpurun_out/conc_$k.json $k
done; done 2>&1 | tee gpurun_out/conc_r06.log
