# Per-tile sweep timelines of the per-step (GPEMU_POTRF=fused) and the group schedule
# (default) (dev tool; the GEMM_TTRACE build from tools/tile_timeline.sh).
set -e
GPEMU_POTRF=fused GPEMU_CHOL_PRIO=0 GPEMU_LIB=gp_emu_uqsa_amd/libgpemu_ttrace.so timeout -k 10 120 python3 tools/tile_timeline.py 127 _fused
GPEMU_CHOL_PRIO=0 GPEMU_LIB=gp_emu_uqsa_amd/libgpemu_ttrace.so timeout -k 10 120 python3 tools/tile_timeline.py 127 _group
rm -f gpurun_out/tile_timeline_*.npy
