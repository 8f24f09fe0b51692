"""mxmoe_amd — MI355X-native (gfx950) mixed-precision MoE GroupGEMM.

Drop-in for the GroupGEMM kernel path of SeaCatComplexes/MxMoE: hand-written CDNA4 HIP kernels
behind a C-ABI (include/mxmoe_gg.h, lib/libmxmoe_gg.so), a Python host mirror of the reference
operator interface, and the reference's run_mxmoe_gg.py / qconfig / tile_config JSON surface.
"""
__version__ = "0.1.0"
