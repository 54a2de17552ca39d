"""recommend-lib_amd — MI355X-native BPR-MF training path (drop-in for the reference's
BPRMFRecommender / util.data_loader.BPRData / util.metrics BPR parts), plus the NCF path of
SURVEY.md §8f (NCFRecommender / NCFData), the Cython rating-SGD models SVD / RSVD
(util/matrix_factorization.pyx) BPR-FM (BPRFMRecommender / BPRFMData) and Item2Vec (Item2VecRecommender SGNS /
BuildCorpus).

The directory name is not a Python identifier; import it with
    importlib.import_module("recommend-lib_amd")
(tests/conftest.py and __graft_entry__.py do exactly that).

Compute lives in libbprmf_amd.so (hand-written HIP for gfx950, C ABI in include/bprmf.h).
"""
from . import _lib
from ._lib import BprmfError
from .build import build, LIB as LIB_PATH
from .data import BPRData
from .model import BPRMF
from . import metrics
from . import sharded
from .sharded import ShardedBPRMF
from . import ncf
from .ncf import NCF, NCFData
from . import ingest
from .ingest import load_rate, load_mat
from . import mf
from .mf import SVD, RSVD, SVDpp
from . import bprfm
from .bprfm import BPRFM, BPRFMData
from . import item2vec
from .item2vec import Item2Vec, SGNS, BuildCorpus, PermutedSubsampledCorpus

BPR = BPRMF  # the reference's class name (BPRMFRecommender.py:28)

__all__ = ["BPRMF", "BPR", "BPRData", "NCF", "NCFData", "ShardedBPRMF", "BprmfError", "metrics",
           "ingest", "load_rate", "load_mat", "SVD", "RSVD", "SVDpp", "BPRFM", "BPRFMData", "Item2Vec", "SGNS", "BuildCorpus",
           "PermutedSubsampledCorpus", "build", "LIB_PATH"]
