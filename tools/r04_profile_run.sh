# round-4 final profile (dev tool): PMC traffic, bench line, rocprofv3 kernel stats
bash tools/round_profile.sh r04
