# the Cholesky's int8 far updates at large n (dev tool): one evaluation's phases with them
# (default from n_pad 32768) and without (GPEMU_OZAKI_FAR_MIN_NP=0), LLH compared
set -o pipefail
mkdir -p gpurun_out
for n in 32768 65536; do
  d=10; [ $n -eq 65536 ] && d=20
  for v in 32768 0; do
    echo "n=$n GPEMU_OZAKI_FAR_MIN_NP=$v"
    GPEMU_OZAKI_FAR_MIN_NP=$v timeout -k 10 300 python3 tools/quick_time.py $n $d || exit 1
  done
done 2>&1 | tee gpurun_out/ozfar_large_r06.log
