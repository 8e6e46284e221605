# round-4 final check after the group-width change (dev tool): the -m gpu suite and
# timings, then the round profile
mkdir -p gpurun_out
bash tools/gpu_check.sh r04w || exit 1
bash tools/round_profile.sh r04w
