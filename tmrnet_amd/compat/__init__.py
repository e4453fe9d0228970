"""Module-name shims for dropping tmrnet_amd into the reference's scripts unchanged.

Put this directory first on sys.path (``sys.path.insert(0, tmrnet_amd.compat.PATH)`` or
``PYTHONPATH=.../tmrnet_amd/compat``); then the reference's own imports
``from NLBlock_MutiConv6_3 import NLBlock, TimeConv`` (train_non-local_mutiConv_resnet.py:24-25),
``from NLBlock import NLBlock`` (train_only_non-local_pretrained.py:23) and ``import models``
(train_memorybank.py:26) resolve to the MI355X implementations.
"""
import os

PATH = os.path.dirname(os.path.abspath(__file__))
