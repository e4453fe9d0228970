"""Shim for code/Training TMRNet/NLBlock_MutiConv6_3.py (NLBlock :10-40, TimeConv :43-79)."""
from tmrnet_amd.nlblock import NLBlock  # noqa: F401
from tmrnet_amd.timeconv import TimeConv  # noqa: F401
