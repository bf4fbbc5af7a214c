"""tempme_amd -- MI355X-native TempME explanation hot path.

Drop-in surface of dharunm236/TempME for the path BASELINE.json names:
  utils.NeighborFinder / RandEdgeSampler / get_null_distribution  -> graph, batch_loader, null_model
  processed.data_preprocess pre_processing / marginal / calculate_edge -> preprocess
  models.TempME (explainer_new.py)                                 -> explainer
  batched device-resident scoring (sampling + encoder + explanation) -> pipeline.ExplainPipeline
Everything computes in libtempme_hip.so (hand-written gfx950 HIP kernels behind the C ABI of
include/tempme.h); importing works without a GPU, calling does not.
"""
from ._lib import SIDE_BGD, SIDE_NONE, SIDE_SRC, SIDE_TGT, SPLIT_NULL, SPLIT_TEST, SPLIT_TRAIN, lib  # noqa: F401
from .batch_loader import RandEdgeSampler  # noqa: F401
from .explainer import TempME  # noqa: F401
from .graph import NeighborFinder, adjacency_from_edges  # noqa: F401
from .null_model import degree_dict, get_null_distribution, load_data_shuffle  # noqa: F401
from .preprocess import calculate_edge, marginal, pre_processing  # noqa: F401

__version__ = "0.1.0"
