"""reference models/ops/modules"""
from .ms_deform_attn import MSDeformAttn, MSDeformAttnCap  # noqa: F401
