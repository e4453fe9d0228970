"""Shim for code/eval/python/NLBlock.py (NLBlock :10-40)."""
from tmrnet_amd.nlblock import NLBlock  # noqa: F401
