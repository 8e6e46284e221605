# LDS bank-conflict cycles of the long-K GEMM for two builds (dev tool): bash tools/pmc_lds.sh libA.so libB.so
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for L in "$@"; do
  for cfg in "64 64 4096 1 1 2" "64 64 4096 0 0 2"; do
    tag=$(echo "$L $cfg" | tr ' .' '__')
    GPEMU_LIB=gp_emu_uqsa_amd/$L timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVE_CYCLES -d gpurun_out/pmc_lds_$tag -o lds --output-format csv -- python3 tools/gemm_one.py $cfg > gpurun_out/pmc_lds_$tag.log 2>&1
  done
done
