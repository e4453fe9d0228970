"""Device-side health word of the train step: failures that kernels can only report on the device
(today: a persistent LSTM launch that gave up a grid barrier and was not recomputed, include/tmr.h
tmr_lstm_status_or) are OR-ed into one int32 per device, stream-ordered and without a host sync.
A give-up on a shared device (another stream or process holding CUs) is normally recovered on
the device by the LSTM's barrier-free solo kernels (csrc/lstm.hip, bit-identical results; the
launch's timeout word then reads 2 and nothing is reported); only with that re-computation
switched off (TMR_LSTM_RECOVER=0, a test hook) does a give-up reach this word.

The fused optimizer kernels (optim.SGD / Adam, tmr_sgd_step_multi / tmr_adam_step_multi) read
the word on the device and skip the update when it is non-zero, so a failed step never changes
the weights.  An inference forward (lstm.LSTM under no_grad) waits and checks at once.
`check()` is called once per optimizer step (optim.SGD / Adam .step()).  It never stalls the
stream: it starts an asynchronous copy of the word into pinned host memory and raises on the value
of the PREVIOUS step's copy once that copy has landed (so a failure surfaces at most one step
later, before the model trains on it for long).  `check(sync=True)` waits for the current stream and checks now
(inference, tests, end of training).  A raised failure clears the word.  Reference counterpart: the LSTM of train_only_non-local_pretrained.py:215,
:230-231, which cannot fail this way on cuDNN.
"""
import torch

from ._lib import call, stream_ptr

_STATE = {}   # device index -> [status (device int32), host copy (pinned), event or None]

LSTM_TIMEOUT = 1


def status_word(device):
    """The device status word (int32, zeroed at creation) kernels OR their failures into."""
    idx = torch.device(device).index or 0
    st = _STATE.get(idx)
    if st is None:
        dev = torch.device("cuda", idx)
        word = torch.empty(1, dtype=torch.int32, device=dev)
        call("tmr_fill_f32", word, 1, 0.0, stream_ptr(dev))   # all-zero bits = int32 0
        st = _STATE[idx] = [word, torch.zeros(1, dtype=torch.int32, pin_memory=True), None]
    return st[0]


def note_lstm(ws):
    """Enqueue status |= (timeout word of the persistent LSTM launch on ws)."""
    call("tmr_lstm_status_or", ws, status_word(ws.device), stream_ptr())


def _raise(v, st):
    """Clear the recorded status (stream-ordered), then raise: a failure is reported once, and a
    later call on a healthy device succeeds."""
    call("tmr_fill_f32", st[0], 1, 0.0, stream_ptr(st[0].device))
    st[1].zero_()
    st[2] = None
    if v & LSTM_TIMEOUT:
        raise RuntimeError("persistent LSTM kernel gave up a grid barrier (its recurrence results "
                           "are invalid) and was not recomputed (TMR_LSTM_RECOVER=0): rerun "
                           "without it, or with TMR_LSTM_PERSIST=0 (per-step path)")
    raise RuntimeError("device status word %#x" % v)


def check(sync=False, device=None):
    """Raise RuntimeError if a device-side failure was recorded (see module doc)."""
    idxs = list(_STATE) if device is None else [torch.device(device).index or 0]
    for idx in idxs:
        st = _STATE.get(idx)
        if st is None:
            continue
        status, host, ev = st
        if sync:
            # .item() waits for the current stream only (the one the kernels were enqueued on),
            # not for the whole device
            v = int(status.item())
            if v:
                _raise(v, st)
            continue
        if ev is not None and ev.query():
            v = int(host.item())
            if v:
                _raise(v, st)
            st[2] = None
        if st[2] is None:
            host.copy_(status, non_blocking=True)
            e = torch.cuda.Event()
            e.record()
            st[2] = e


def reset(device=None):
    """Clear the recorded status (tests)."""
    for idx, st in list(_STATE.items()):
        if device is None or idx == (torch.device(device).index or 0):
            torch.cuda.synchronize(st[0].device)
            st[0].zero_()
            st[1].zero_()
            st[2] = None
