# Per-tile timeline of the whole fused-Cholesky sweep (dev tool), panel tiles last
# (default) and at list position 512 (GPEMU_PANEL_POS).
set -e
GPEMU_CHOL_PRIO=0 GPEMU_LIB=gp_emu_uqsa_amd/libgpemu_ttrace.so timeout -k 10 120 python3 tools/tile_timeline.py 127 _default
GPEMU_PANEL_POS=512 GPEMU_CHOL_PRIO=0 GPEMU_LIB=gp_emu_uqsa_amd/libgpemu_ttrace.so timeout -k 10 120 python3 tools/tile_timeline.py 127 _pos512
