"""tmrnet_amd: TMRNet's per-clip train-step hot path, MI355X-native (HIP/CDNA4 kernels in
libtmr.so behind a C ABI, PyTorch-ROCm only for memory, streams and torch.distributed)."""
from . import _lib, ops  # noqa: F401
from .lstm import LSTM  # noqa: F401
from .nlblock import NLBlock, LFBRows  # noqa: F401
from .trunk import ResNet50Share, resnet50_share  # noqa: F401
from .model import resnet_lstm, resnet_lstm_LFB, MemoryBankModel  # noqa: F401
from .loss import CrossEntropyLoss  # noqa: F401
from .optim import SGD, Adam  # noqa: F401

__version__ = "0.1.0"
