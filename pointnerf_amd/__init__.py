"""pointnerf_amd -- MI355X-native Point-NeRF hot path.

The world-coordinate neural-point query, K-neighbour gather + aggregation MLP
and ray-march composite of yjcaimeow/pointnerf, as hand-written HIP kernels for
gfx950 behind the C ABI in include/pnr.h (libpnr.so), with Python drop-ins for
the reference's querier / PointAggregator / ray_march / NeuralPointsRayMarching
seams; autograd through the same kernels for the finetune step (train.py), a
bf16-MFMA aggregation mode, reference-format checkpoints and the fork's 2-D
neural renderer.  See DESIGN.md.
"""
from . import _lib  # noqa: F401  (loads torch before libpnr.so)
from .aggregator import PointAggregator, frag_pack, frag_unpack  # noqa: F401
from .options import lego_opt  # noqa: F401
from .querier import lighting_fast_querier, ray_mid_t, hyperparameters_from_bbox  # noqa: F401
from .ray_march import ray_march, radiance_render, alpha_blend, no_tone_map  # noqa: F401
from .renderer import NeuralPoints, NeuralPointsRayMarching, RenderGraph  # noqa: F401
from .voxelize import construct_vox_points_closest  # noqa: F401
from .neural_render import NeuralRenderer  # noqa: F401
from .checkpoint import load_ray_marching, save_ray_marching, prune, grow_points  # noqa: F401
from .aggregator import frag_pack_bf16  # noqa: F401

__version__ = "0.1.0"
