# Micro-benchmarks of the diagonal factor (dev tool): the leaf probe and the stand-alone
# 128 x 128 factor + inverse per variant (tools/hip/*_bin, db_bench_*).
mkdir -p gpurun_out
for b in tools/hip/leaf_probe_bin tools/hip/db_bench_*; do
  [ -x "$b" ] || continue
  echo "== $b"; timeout -k 5 60 "$b" || exit 1
done
