"""iddgcn_amd — MI355X-native hot path of IDDGCN (AhauBioinformatics/IDDGCN).

The directed multi-relational graph convolution of prediction/IDDGCN.py,
forward and backward, as hand-written HIP kernels for gfx950 behind a C-ABI
(include/iddgcn.h, libiddgcn_hip.so), driven from a Keras-shaped Python
surface:

    from iddgcn_amd import get_IDDGCN_Model, get_adj_mats, Adam, BinaryCrossentropy
"""
from ._lib import IddgcnError  # noqa: F401
from .graph import get_adj_mats  # noqa: F401
from .model import (Adam, BinaryCrossentropy, DistMult, IDDGCN_Layer, IDDGCN_Model,  # noqa: F401
                    SaveWeightsCallback, get_IDDGCN_Model)
from .utils import generate_reverse_triplets, get_y_true  # noqa: F401
from . import explain  # noqa: F401,E402  (explaiNE / GNNExplainer / IDDGCN explainer on the HIP path)
from . import similarity  # noqa: F401,E402  (feat_similarity.py similarity graph on MFMA)
