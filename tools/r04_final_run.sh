# round-4 final check (dev tool): the -m gpu suite and timings of the head, then the
# round profile (PMC traffic, bench line, rocprofv3 kernel stats)
mkdir -p gpurun_out
bash tools/gpu_check.sh r04z || exit 1
bash tools/round_profile.sh r04z
