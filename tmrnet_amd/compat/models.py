"""Shim for code/models.py: ``resnet_lstm(args, num_class)`` with ``get_optimizers()``.

Keys follow the reference file: ``res.0.weight`` ... (Sequential of resnet50 children,
models.py:26-28), ``lstm.*``, ``fc.*``.  forward follows the working memory-bank model of
Training memory bank model/train_singlenet_phase_1fc.py:223-232 (the shipped models.py:38-48
feeds a 5-D tensor to Conv2d and raises): x (B,T,3,224,224) or (F,3,224,224) -> (F, num_class);
the caller keeps outputs[T-1::T] (train_memorybank.py:262).
"""

from tmrnet_amd.model import MemoryBankModel
from tmrnet_amd.optim import SGD, Adam


class resnet_lstm(MemoryBankModel):  # noqa: N801  (reference name)
    def __init__(self, args, num_class):
        seq = getattr(args, "num_frames", None) or getattr(args, "seq", None) or 10
        super().__init__(seq_len=int(seq), num_classes=num_class, indexed_trunk=True)
        self.args = args

    def forward(self, x):
        # T from a 5-D (B,T,3,224,224) input, passed down per call: writing it into the module
        # would race between threads driving one instance (SURVEY.md §8b Threading)
        return super().forward(x, seq_len=x.shape[1] if x.dim() == 5 else None)

    def get_optimizers(self):
        """models.py:50-69: res at lr/10, lstm and fc at lr; opt 0 = SGD, 1 = Adam."""
        a = self.args
        groups = [{"params": self.res.parameters()},
                  {"params": self.lstm.parameters(), "lr": a.lr},
                  {"params": self.fc.parameters(), "lr": a.lr}]
        if a.opt == 0:
            return SGD(groups, lr=a.lr / 10, momentum=a.momentum, dampening=a.dampening,
                       weight_decay=a.weightdecay, nesterov=a.nesterov)
        if a.opt == 1:
            return Adam(groups, lr=a.lr / 10)
        return None
