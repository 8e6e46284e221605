# Column-group widths at n=65536, d=20 (config C4 on one GPU) (dev tool, GPU box).
for w in "4:80,2:40" "8:160,4:80,2:40" "16:256,8:128,4:64,2:32"; do
  printf "%-26s " "$w"
  GPEMU_POTRF_W="$w" timeout -k 10 200 python3 tools/quick_time.py 65536 20 | grep phases | python3 -c "import sys,ast; l=sys.stdin.read(); d=ast.literal_eval(l[l.index('{'):]); print(' '.join('%s %.0f' % (k, v) for k, v in d.items()))"
done
