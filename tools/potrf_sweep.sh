# Sweep the fused Cholesky's column-group widths (GPEMU_POTRF_W) at n=16384 (dev tool, GPU box).
set -e
for w in "4:80,2:40" "4:80" "4:64" "4:96,2:64" "8:96,4:64" "4:100" "2:64" "4:48" "8:100,4:80" "4:88,2:72" "1:0"; do
  printf "%-16s " "$w"
  GPEMU_POTRF_W="$w" timeout -k 10 120 python3 tools/quick_time.py 16384 10 | grep phases | python3 -c "import sys,ast; l=sys.stdin.read(); d=ast.literal_eval(l[l.index('{'):]); print('chol %.2f total %.2f' % (d['cholesky'], d['total']))"
done
