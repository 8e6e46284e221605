# round-5 final check (dev tool), in two gpurun calls:
#   bash tools/r05_final_run.sh check   -- the -m gpu suite and timings of the head (gpu_check.sh)
#   bash tools/r05_final_run.sh profile -- smoke(), then the round profile (PMC traffic, bench line,
#                                          rocprofv3 kernel stats; round_profile.sh)
set -o pipefail
mkdir -p gpurun_out
case "$1" in
  check) bash tools/gpu_check.sh ${2:-r05z} ;;
  profile)
    timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r05.log 2>&1 || exit 1
    tail -2 gpurun_out/smoke_r05.log
    bash tools/round_profile.sh r05 ;;
  *) echo "usage: $0 check|profile"; exit 2 ;;
esac
