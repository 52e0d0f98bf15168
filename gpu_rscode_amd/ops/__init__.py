"""Device ops: GF-GEMM, Gauss-Jordan inverse, coding matrices, synthetic data."""
from .gemm import Gemm16Plan, GemmPlan, build_desc, desc_layout, gf_gemm, pad_m, perm_tables_from_coeff, tile_for
from .inverse import PatternDecoder, decode_system16_into_plan, decode_system_into_plan, gf_invert, invert_into_plan
from .matrix import decode_matrix, encoding_matrix, gen_matrix_device, generator
from .random import fill_random_

__all__ = [
    "GemmPlan", "Gemm16Plan", "build_desc", "desc_layout", "gf_gemm", "pad_m", "tile_for", "perm_tables_from_coeff",
    "PatternDecoder", "gf_invert", "invert_into_plan", "decode_system_into_plan", "decode_system16_into_plan", "decode_matrix", "encoding_matrix",
    "gen_matrix_device", "generator",
    "fill_random_",
]
