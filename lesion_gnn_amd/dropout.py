"""Dropout on the HIP path: masks from the counter-based generator of lgnn_dropout_masks, applied
inside the consuming kernels (GATConv attention, the GIN MLP) or by lgnn_mask_mul (between convs).

Replaces torch's Bernoulli draws in the reference's dropout sites: nn.Dropout between GIN convs
(src/lesion_gnn/models/gin.py:27,32), PyG MLP's dropout after BatchNorm + ELU (gin.py:23) and
GATConv's attention dropout (gat.py:31). Semantics are torch's (keep with probability 1 - p,
kept values scaled by 1 / (1 - p)); the random stream is this package's own: every mask is a pure
function of (seed, counter, stream, element) — see include/lgnn.h — so the CPU oracle
(oracle/pyg_ref.py DropoutMasks) regenerates exactly the masks a step used.

A model draws all masks of its forward in ONE launch from its generator state: a non-persistent
buffer `_dropout_rng` (uint64 [seed, counter, ticket words...] x 8, stored as int64; not in state_dict, so
checkpoint keys stay PyG's; moved by .to(device)). The seed is derived from the state of torch's default
generator (set by torch.manual_seed, advanced by weight init) WITHOUT drawing from it — so building a model does not shift the random stream later
draws (weight init of other modules, data shuffling, splits) see. The launch advances the counter
on the device, so captured HIP graphs draw fresh masks per replay. A resumed run restarts the
counter (the state is not checkpointed, to keep the reference's state_dict keys): masks differ
from an uninterrupted run's, as torch's own dropout stream does after a resume.
"""
from __future__ import annotations

import ctypes
import math

import torch

from . import _lib

MAX_MASKS = 16  # LGNN_MAX_MASKS


STATE_WORDS = 8  # uint64: seed, counter, then the launch's ticket words (lgnn.h)


_M64 = 2 ** 64 - 1


def _splitmix64(z: int) -> int:
    z = (z + 0x9E3779B97F4A7C15) & _M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    return z ^ (z >> 31)


_UNSALTED = [0]  # unsalted seeds derived so far in this process


def param_salt(module) -> bytes | None:
    """The digest of a freshly built module's initial parameters (None when any parameter has no
    data: meta device, lazy modules)."""
    import hashlib

    h = hashlib.sha256()
    for p in module.parameters():
        if p.is_meta or isinstance(p, torch.nn.parameter.UninitializedParameter):
            return None
        h.update(p.detach().to("cpu", torch.float32).contiguous().numpy().tobytes())
    return h.digest()


def derived_seed(salt: bytes | None = None) -> int:
    """A seed derived from torch's default CPU generator WITHOUT advancing it: the splitmix64 of a
    hash of its current state (read, not drawn from) and of a salt.

    Models pass the digest of their initial parameters (`param_salt`), so the seed is a function
    of the generator state and the model's own initial weights only: `torch.manual_seed(s);
    m1 = Model(); torch.manual_seed(s); m2 = Model()` gives m1 and m2 the same dropout stream (as
    torch's own dropout would), whatever was built earlier in the process, and two models whose
    weights differ (CPU or GPU init) get different streams. Without a salt (a lone conv, meta
    parameters) a per-process counter is mixed in instead, so two such constructions with no
    generator draw between them still differ. Building a model leaves the generator's stream
    exactly where weight init left it."""
    import hashlib

    if salt is None:
        n = _UNSALTED[0]
        _UNSALTED[0] += 1
        salt = b"unsalted" + n.to_bytes(8, "little")
    state = torch.default_generator.get_state().numpy().tobytes()
    h = int.from_bytes(hashlib.sha256(state + salt).digest()[:8], "little")
    return _splitmix64(h) & (2 ** 62 - 1)


def new_state(seed: int | None = None, salt: bytes | None = None) -> torch.Tensor:
    """A generator state [seed, counter = 0, tickets = 0 ...] (CPU; register it as a buffer)."""
    if seed is None:
        seed = derived_seed(salt)
    return torch.tensor([int(seed)] + [0] * (STATE_WORDS - 1), dtype=torch.int64)


def set_state(state: torch.Tensor, seed: int, counter: int = 0) -> None:
    """Position a generator state (tests: the oracle regenerates the masks from (seed, counter))."""
    state.copy_(torch.tensor([int(seed), int(counter)] + [0] * (STATE_WORDS - 2),
                             dtype=torch.int64))


def get_state(state: torch.Tensor) -> tuple[int, int]:
    """(seed, counter) of a state (synchronises)."""
    s = state.cpu().tolist()
    return s[0] & (2 ** 64 - 1), s[1] & (2 ** 64 - 1)


def threshold_scale(p: float) -> tuple[int, float]:
    """(thr, scale): keep element i when its 24 random bits are >= thr = floor(p * 2^24); kept
    values are multiplied by scale = fp32(1 / (1 - p)), rounded to fp32 (nearest, ties to even)
    in plain Python arithmetic: a torch scalar here was a `Tensor.item()` graph break under
    torch.compile (the reference experiment compiles its model with dropout 0.35)."""
    if not 0.0 <= p < 1.0:
        raise ValueError(f"dropout probability must be in [0, 1), got {p}")
    m, e = math.frexp(1.0 / (1.0 - p))  # 1 / (1 - p) >= 1: a normal fp32 number
    return int(p * 16777216.0), math.ldexp(round(m * 16777216.0), e - 24)


def key(module, p: float) -> str:
    """The constant-string form of a module's dropout probability p for masks(): refreshed from
    p in eager mode (so a changed `dropout.p` takes effect), read as traced under compile, where
    p itself would be a symbolic float."""
    if not torch.compiler.is_compiling():
        module._dropout_key = repr(float(p))
    return module._dropout_key


_GLOBAL: dict = {}


def global_state(device) -> torch.Tensor:
    """A per-device generator for dropout sites used outside a model (a lone conv module)."""
    dev = torch.device(device)
    key = (dev.type, dev.index)
    st = _GLOBAL.get(key)
    if st is None:
        st = _GLOBAL[key] = new_state().to(dev)
    return st


def masks(state: torch.Tensor, shapes: list, p: float | str) -> list[torch.Tensor]:
    """One fp32 mask per shape (0 or 1 / (1 - p)), mask j from stream j, in one launch; the
    state's counter advances by one. p may be given as its repr (a module's `dropout_key`):
    under torch.compile(dynamic=True) a float module attribute is traced as a symbolic float,
    which the op's threshold / scale arguments cannot take, while a string stays a constant."""
    if len(shapes) > MAX_MASKS:
        raise ValueError(f"at most {MAX_MASKS} masks per launch")
    thr, scale = threshold_scale(float(p))
    numels = []
    for s in shapes:
        n = 1
        for d in s:
            n *= d
        numels.append(n)
    if torch.compiler.is_compiling():
        from . import library  # noqa: F401  (registers torch.ops.lgnn.*)

        flat = torch.ops.lgnn.dropout_masks(state, numels, thr, scale)
    else:
        flat = dropout_masks_raw(state, numels, thr, scale)
    out, off = [], 0
    for n, s in zip(numels, shapes):
        out.append(flat[off:off + n].view(*s))
        off += _pad4(n)
    return out


def _pad4(n):
    return (n + 3) // 4 * 4


def dropout_masks_raw(state: torch.Tensor, numels: list, thr: int, scale: float) -> torch.Tensor:
    """All masks in one flat fp32 allocation (mask j at the sum of the earlier masks' sizes,
    each rounded up to 4 elements: 16-B aligned), drawn by one lgnn_dropout_masks launch."""
    _lib.require_gpu(state)
    if state.dtype != torch.int64 or state.numel() != STATE_WORDS or not state.is_contiguous():
        raise _lib.LgnnError("dropout generator state must be a contiguous int64 [8] tensor")
    dev = state.device
    offs, tot = [], 0
    for n in numels:
        offs.append(tot)
        tot += _pad4(int(n))
    flat = torch.empty(tot, dtype=torch.float32, device=dev)
    k = len(numels)
    base = flat.data_ptr()
    _lib.call("lgnn_dropout_masks", k, (ctypes.c_void_p * k)(*[base + 4 * o for o in offs]),
              (ctypes.c_int64 * k)(*[int(n) for n in numels]),
              (ctypes.c_uint32 * k)(*([thr] * k)), (ctypes.c_float * k)(*([scale] * k)),
              state.data_ptr(), 1, _lib.stream(dev))
    return flat


def _mul(x: torch.Tensor, m: torch.Tensor) -> torch.Tensor:
    _lib.require_gpu(x, m)
    if x.dtype != torch.float32 or m.dtype != torch.float32 or x.shape != m.shape:
        raise _lib.LgnnError("mask_mul: fp32 tensors of one shape")
    x, m = x.contiguous(), m.contiguous()
    y = torch.empty_like(x)
    _lib.call("lgnn_mask_mul", _lib.ptr(x), _lib.ptr(m), _lib.ptr(y), x.numel(),
              _lib.stream(x.device))
    return y


class _MaskMul(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, m):
        ctx.save_for_backward(m)
        return _mul(x, m)

    @staticmethod
    def backward(ctx, dy):
        (m,) = ctx.saved_tensors
        return _mul(dy, m), None


def mask_mul(x: torch.Tensor, m: torch.Tensor) -> torch.Tensor:
    """x * m (the dropout product; backward dy * m) on lgnn_mask_mul."""
    if torch.compiler.is_compiling():
        from . import library  # noqa: F401

        return torch.ops.lgnn.mask_mul(x, m)
    return _MaskMul.apply(x, m)
