"""The module-name shims resolve and keep the reference's parameter names (no GPU needed)."""
import sys
from types import SimpleNamespace as NS

import tmrnet_amd.compat as compat


def test_shims_import_and_keys():
    sys.path.insert(0, compat.PATH)
    try:
        import NLBlock_MutiConv6_3 as m1
        import NLBlock as m2
        import models
    finally:
        sys.path.remove(compat.PATH)
    nl = m1.NLBlock()
    assert sorted(k for k, _ in nl.named_parameters()) == sorted(
        ["linear%d.%s" % (i, t) for i in range(1, 5) for t in ("weight", "bias")] +
        ["layer_norm.weight", "layer_norm.bias"])
    assert tuple(nl.layer_norm.weight.shape) == (1, 512)
    tc = m1.TimeConv()
    assert tuple(tc.timeconv3.weight.shape) == (512, 512, 7)
    assert m2.NLBlock is m1.NLBlock
    args = NS(num_frames=10, opt=0, lr=5e-4, momentum=0.9, dampening=0, weightdecay=5e-4,
              nesterov=False)
    m = models.resnet_lstm(args, 6)
    keys = list(m.state_dict())
    assert keys[0] == "res.0.weight" and "res.4.0.conv1.weight" in keys and "fc.weight" in keys
    opt = m.get_optimizers()
    assert len(opt.param_groups) == 3
    assert opt.param_groups[0]["lr"] == 5e-5 and opt.param_groups[1]["lr"] == 5e-4
