# round-4 A/B (dev tool): column-group widths of the fused Cholesky (GPEMU_POTRF_W) at the
# head -- the lone evaluation's phases at n = 16384 and 4096 and the two-try bench;
# alternating, twice
mkdir -p gpurun_out
for rep in 1 2; do
  for W in "4:80,2:40" "4:40" "4:48,2:24" "8:80,4:40"; do
    echo "== W=$W rep $rep"
    for n in 16384 8192; do GPEMU_POTRF_W=$W timeout -k 10 120 python3 tools/quick_time.py $n 10 | grep -v "^gemm" | cut -c1-200 || exit 1; done
    GPEMU_POTRF_W=$W timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline \
      --no-other-configs --no-profile 2>/dev/null | tail -1 | cut -c1-160 || exit 1
  done
done > gpurun_out/width_ab_r04.log 2>&1
