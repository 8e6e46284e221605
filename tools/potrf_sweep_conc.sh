# Column-group widths (GPEMU_POTRF_W) under the default bench (two tries in flight) (dev tool, GPU box).
for w in "4:80,2:40" "8:64,4:32" "8:80,4:40" "8:48" "8:96,4:48,2:24" "16:80,8:40" "4:0"; do
  printf "%-18s " "$w"
  GPEMU_POTRF_W="$w" timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-profile --steps 8 | python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('%.3f evals/s' % d['value'])"
done
