"""Checkpoints: the reference's ``state_dict`` files, both trunk namespaces.

The reference saves ``model.module.state_dict()`` / ``best_model_wts`` with ``torch.save``
(e.g. ``Training TMRNet/train_only_non-local_pretrained.py:900-903``) and loads them with
``load_state_dict(torch.load(path), strict=False)`` (:554, :625; ``train_non-local_mutiConv_resnet.py``
:707, :774), strict only in eval (``eval/python/..._mutiConv6_3.py:429``).  Two trunk namespaces
exist: the inline scripts' ``share.{conv1,bn1,layer1..4}`` and ``code/models.py:26-28``'s
``res.{0,1,4,5,6,7}`` (``Sequential(*list(resnet50().children())[:-1])``).  Loading one into the
other with ``strict=False`` silently keeps the random trunk; here the namespace is mapped and every
key that is still dropped is reported (warning, or an error with ``strict=True``).

Loading uses ``torch.load(..., weights_only=True)`` only.
"""
import warnings

import torch

# torchvision resnet50 children order (code/models.py:26-28 keeps [:-1])
_SHARE_TO_RES = {"conv1": "0", "bn1": "1", "relu": "2", "maxpool": "3", "layer1": "4",
                 "layer2": "5", "layer3": "6", "layer4": "7", "avgpool": "8"}
_RES_TO_SHARE = {v: k for k, v in _SHARE_TO_RES.items()}


class CheckpointKeyWarning(UserWarning):
    pass


def _strip_module(sd):
    """DataParallel/DDP wrappers prefix keys with 'module.'."""
    if sd and all(k.startswith("module.") for k in sd):
        return {k[len("module."):]: v for k, v in sd.items()}
    return dict(sd)


def convert_trunk_namespace(sd, to):
    """Rename trunk keys between 'share.<child>.*' (inline scripts) and 'res.<index>.*'
    (code/models.py).  Other keys are kept."""
    if to not in ("share", "res"):
        raise ValueError("to must be 'share' or 'res'")
    out = {}
    for k, v in sd.items():
        parts = k.split(".")
        if to == "res" and parts[0] == "share" and len(parts) > 1 and parts[1] in _SHARE_TO_RES:
            k = ".".join(["res", _SHARE_TO_RES[parts[1]]] + parts[2:])
        elif to == "share" and parts[0] == "res" and len(parts) > 1 and parts[1] in _RES_TO_SHARE:
            k = ".".join(["share", _RES_TO_SHARE[parts[1]]] + parts[2:])
        out[k] = v
    return out


def _trunk_namespace(model_keys):
    if any(k.startswith("share.") for k in model_keys):
        return "share"
    if any(k.startswith("res.") for k in model_keys):
        return "res"
    return None


def load_checkpoint(model, src, strict=False, map_location="cpu"):
    """Load a reference checkpoint (path or state_dict) into `model`.

    Strips a 'module.' prefix, maps the trunk namespace to the model's, then loads.  Keys the
    model does not take and model keys the file lacks are reported with a CheckpointKeyWarning
    (strict=False, the reference's training default) or raise (strict=True).  Returns
    (missing_keys, unexpected_keys)."""
    sd = torch.load(src, map_location=map_location, weights_only=True) if isinstance(src, str) \
        else src
    sd = _strip_module(sd)
    ns = _trunk_namespace(model.state_dict().keys())
    if ns is not None:
        sd = convert_trunk_namespace(sd, ns)
    res = model.load_state_dict(sd, strict=False)
    missing, unexpected = list(res.missing_keys), list(res.unexpected_keys)
    if missing or unexpected:
        msg = ("checkpoint/model key mismatch: %d model keys not in the checkpoint (kept at their "
               "current values)%s; %d checkpoint keys not used by the model%s"
               % (len(missing), (": " + ", ".join(missing[:8]) + (" ..." if len(missing) > 8 else ""))
                  if missing else "", len(unexpected),
                  (": " + ", ".join(unexpected[:8]) + (" ..." if len(unexpected) > 8 else ""))
                  if unexpected else ""))
        if strict:
            raise RuntimeError(msg)
        warnings.warn(msg, CheckpointKeyWarning, stacklevel=2)
    return missing, unexpected


def save_checkpoint(model, path, namespace=None):
    """torch.save of the state_dict (the reference's format); namespace='res'/'share' writes the
    other script family's trunk key names."""
    sd = model.state_dict()
    if namespace is not None:
        sd = convert_trunk_namespace(sd, namespace)
    torch.save(sd, path)
