# round-4 A/B (dev tool): schedule switches at the head -- two-try bench under auto / group /
# fused, and the lone evaluation's Cholesky under group chain strides; alternating, twice
mkdir -p gpurun_out
for rep in 1 2; do
  for S in auto group fused; do
    echo "== bench POTRF=$S rep $rep"
    GPEMU_POTRF=$S timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline \
      --no-other-configs --no-profile 2>/dev/null | tail -1 | cut -c1-160 || exit 1
  done
  for ST in 896 600 1300; do
    echo "== stride $ST rep $rep"
    GPEMU_GROUP_STRIDE=$ST timeout -k 10 120 python3 tools/quick_time.py 16384 10 | grep -v "^gemm" | cut -c1-200 || exit 1
  done
done > gpurun_out/env_ab_r04.log 2>&1
