"""MI355X-native multi-scale temporal deformable attention (MSDA) for the
SAGA-DVC/multimodal-feature-learning deformable DVC path.

Layout:
  csrc/msda.hip        HIP kernels (gfx950) + the extern "C" entry points of include/msda_hip.h
  lib/libmsda_hip.so   built by __graft_entry__.build()
  _native.py           ctypes binding of the C-ABI (no fallback)
  msda.py              host checks, layout normalisation, autograd.Function
  MultiScaleDeformableAttention.py   mirror of the reference's pybind extension API
  models/...           mirror of the reference modules on the path (same names / signatures)
  utils/dam.py         Sparse-DETR decoder attention map (HIP scatter kernel)
  train_step.py        flat-gradient data-parallel step, HIP-graph captured (bench.py)

The directory name is not a Python identifier; import it with
``importlib.import_module("multimodal-feature-learning_amd")``.  The import registers
``mfl_amd`` (and ``mfl_amd.<submodule>``) as aliases of the same module objects.
"""
import os as _os
import sys as _sys

# HIP runtime setting, read once when the process initialises HIP (so it must be set before the
# first device call): with the CLR's graph packet capture (the default), a captured bf16 training
# step replayed after eager work that allocates device memory produced corrupted gradients
# (tools/step_diag.py --graph 1; exact again with the capture off).  Replays
# with nothing allocating between them were exact either way.
_PACKET_CAPTURE_VAR = "DEBUG_CLR_GRAPH_PACKET_CAPTURE"
import torch as _torch  # noqa: E402  (importing torch does not initialise HIP)
# HIP already up when the package was imported: the variable counts only if it was set by then
_HIP_UP_AT_IMPORT = _torch.cuda.is_initialized()
_PACKET_CAPTURE_AT_IMPORT = _os.environ.get(_PACKET_CAPTURE_VAR)
_os.environ.setdefault(_PACKET_CAPTURE_VAR, "0")
# Read when a ProcessGroupNCCL is constructed: its per-device event cache hands the end event of a
# collective captured in a HIP graph to a later eager collective; kept off, so an event the RCCL watchdog
# polls has only ever been recorded on the eager collectives' stream (train_step._capture_group)
_EVENT_CACHE_VAR = "TORCH_NCCL_CUDA_EVENT_CACHE"
_os.environ.setdefault(_EVENT_CACHE_VAR, "0")


def graph_packet_capture_off():
    """True when the HIP runtime of this process runs with the graph packet capture off: the
    variable is "0" now, and it was already "0" when HIP initialised (the package set it, HIP
    initialising after the import; or the environment had it before HIP came up)."""
    if _os.environ.get(_PACKET_CAPTURE_VAR) != "0":
        return False
    return (not _HIP_UP_AT_IMPORT) or _PACKET_CAPTURE_AT_IMPORT == "0"

__version__ = "0.1.0"

from . import _native  # noqa: E402
from . import _trace  # noqa: E402,F401
from . import msda  # noqa: E402
from . import MultiScaleDeformableAttention  # noqa: E402
from . import models  # noqa: E402
from .models.modules import attention, embedding_layers, misc_modules  # noqa: E402,F401
from .models import base_encoder  # noqa: E402,F401
from .models.deformable import unimodal_deformable_transformer  # noqa: E402,F401
from .models.deformable import multimodal_deformable_transformer  # noqa: E402,F401
from .models.sparse import unimodal_sparse_deformable_transformer  # noqa: E402,F401
from .models.ops.functions import ms_deform_attn_func  # noqa: E402,F401
from .models.ops.modules import ms_deform_attn  # noqa: E402,F401
from . import utils  # noqa: E402,F401
from .utils import dam, box_ops, preds_postprocess  # noqa: E402,F401
from .models import matcher, load_weights, dvc_common  # noqa: E402,F401
from .models.modules import layers  # noqa: E402,F401
from .models import unimodal_caption_decoder, multimodal_caption_decoder  # noqa: E402,F401
from .models.deformable import unimodal_deformable_dvc, multimodal_deformable_dvc  # noqa: E402,F401
from .models.sparse import unimodal_sparse_dvc  # noqa: E402,F401
from . import dvc_core  # noqa: E402,F401
from . import train_step  # noqa: E402,F401

ALIAS = "mfl_amd"


def _register_alias():
    prefix = __name__ + "."
    _sys.modules.setdefault(ALIAS, _sys.modules[__name__])
    for name, mod in list(_sys.modules.items()):
        if name.startswith(prefix):
            _sys.modules.setdefault(ALIAS + "." + name[len(prefix):], mod)


_register_alias()
