# round-4 A/B (dev tool): column-group widths of the row-block objective (GPEMU_DIST_W) at
# P = 1 and 2 (loopback), n = 16384; alternating, twice
mkdir -p gpurun_out
for rep in 1 2; do
  for W in "8:160,4:80,2:40" "4:48,2:24" "8:96,4:48,2:24"; do
    for P in 1 2; do
      echo "== W=$W P=$P rep $rep"
      GPEMU_DIST_W=$W timeout -k 10 240 python3 tools/dist_objective.py --loopback $P --points 16384 --dims 10 --grad | cut -c1-200 || exit 1
    done
  done
done > gpurun_out/distw_ab_r04.log 2>&1
