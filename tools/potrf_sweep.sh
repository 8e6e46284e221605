# Sweep the fused Cholesky's column-group widths (GPEMU_POTRF_W) at n=16384 (dev tool, GPU box).
set -e
for w in ${POTRF_WIDTHS:-"4:80,2:40" "1:127,4:80,2:40" "2:126,4:80,2:40" "1:127,2:125,4:80,2:40" "1:127,8:96,4:64,2:32"}; do
  printf "%-24s " "$w"
  GPEMU_POTRF_W="$w" timeout -k 10 120 python3 tools/quick_time.py 16384 10 | grep phases | python3 -c "import sys,ast; l=sys.stdin.read(); d=ast.literal_eval(l[l.index('{'):]); print('chol %.2f total %.2f' % (d['cholesky'], d['total']))"
done
