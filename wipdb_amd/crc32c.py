"""Python mirror of WipDB's crc32c surface and of the batch engine.

Per-span functions mirror ``kv::crc32c`` (/root/reference/kv/src/util/crc32c.h):
``extend`` (:24), ``value`` (:27-29), ``mask`` (:38-41), ``unmask`` (:44-47),
``MASK_DELTA`` (:31), ``is_fast_crc32_supported`` (:19).  They run the
library's host CPU path (crc32c_cpu.cc), as the reference's do.

``Engine`` is the batch boundary: one context per GPU, spans handed to the
gfx950 kernels through the C-ABI.  Inputs are either numpy arrays in host
memory (staged through pinned buffers) or torch tensors already resident
on the context's device (asynchronous, on the caller's stream).  Nothing
here falls back to the CPU: a HIP failure raises ``HcrcError``.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence

import numpy as np

from . import _lib
from ._lib import (HCRC_BALANCE, HCRC_DEVICE_PTRS, HCRC_MASK_OUTPUT, HCRC_PACKED, HCRC_SPLIT_LONG,
                   HCRC_SPLIT_SMALL, HcrcError, check)

MASK_DELTA = 0xA282EAD8


def _ptr(a) -> int:
    if a is None:
        return 0
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    return int(a.data_ptr())  # torch tensor


def _as_bytes(data) -> np.ndarray:
    if isinstance(data, np.ndarray):
        return np.ascontiguousarray(data).view(np.uint8).reshape(-1)
    return np.frombuffer(bytes(data), dtype=np.uint8)


# --------------------------------------------------------------------------
# per-span surface (host CPU path), kv/src/util/crc32c.h
# --------------------------------------------------------------------------
def extend(init_crc: int, data) -> int:
    """crc32c of concat(A, data) given init_crc = crc32c(A) (crc32c.h:21-24)."""
    buf = _as_bytes(data)
    return int(_lib.load().hcrc_cpu_extend(init_crc & 0xFFFFFFFF, _ptr(buf), buf.size))


def value(data) -> int:
    """crc32c of data (crc32c.h:27-29)."""
    return extend(0, data)


def mask(crc: int) -> int:
    """Rotate right 15, add kMaskDelta (crc32c.h:38-41)."""
    crc &= 0xFFFFFFFF
    return (((crc >> 15) | (crc << 17)) + MASK_DELTA) & 0xFFFFFFFF


def unmask(masked_crc: int) -> int:
    """Inverse of mask (crc32c.h:44-47)."""
    rot = (masked_crc - MASK_DELTA) & 0xFFFFFFFF
    return ((rot >> 17) | (rot << 15)) & 0xFFFFFFFF


def is_fast_crc32_supported() -> str:
    """Same strings as crc32c.cc:467-492."""
    return "Supported on x86" if _lib.load().hcrc_cpu_is_accelerated() else "Not supported on x86"


def cpu_batch(base: np.ndarray, offsets, lengths, inits=None, mask_output=False,
              threads: int = 1) -> np.ndarray:
    """Host CPU batch (the library's own SSE4.2 path) -- not the GPU path."""
    base = _as_bytes(base)
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    ln = np.ascontiguousarray(lengths, dtype=np.uint32)
    ini = None if inits is None else np.ascontiguousarray(inits, dtype=np.uint32)
    out = np.empty(off.size, dtype=np.uint32)
    flags = HCRC_MASK_OUTPUT if mask_output else 0
    check(_lib.load().hcrc_cpu_batch(_ptr(base), _ptr(off), _ptr(ln), _ptr(ini), _ptr(out),
                                     off.size, flags, threads), "hcrc_cpu_batch")
    return out


def device_count() -> int:
    n = ctypes.c_int(0)
    rc = _lib.load().hcrc_device_count(ctypes.byref(n))
    return n.value if rc == 0 else 0


# --------------------------------------------------------------------------
# batch engine (GPU)
# --------------------------------------------------------------------------
def _check_tensor(t, name: str, device, dtypes, min_numel: int = 0) -> None:
    """Device tensor arguments are raw pointers at the C-ABI: a wrong dtype
    (e.g. torch's default int64 for a u32 column), a strided view or a tensor
    on another device would be read as garbage or out of bounds by the
    kernel, so they are rejected here."""
    if t is None:
        return
    if not hasattr(t, "data_ptr"):
        raise TypeError(f"{name}: expected a torch tensor")
    if t.device != device:
        raise ValueError(f"{name}: on {t.device}, the engine's device is {device}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: must be contiguous")
    if dtypes is not None and t.dtype not in dtypes:
        raise TypeError(f"{name}: dtype {t.dtype}, expected one of {[str(d) for d in dtypes]}")
    if t.numel() < min_numel:
        raise ValueError(f"{name}: {t.numel()} elements, need {min_numel}")


def _dtypes():
    import torch
    u32 = tuple(d for d in (torch.int32, getattr(torch, "uint32", None)) if d is not None)
    u64 = tuple(d for d in (torch.int64, getattr(torch, "uint64", None)) if d is not None)
    return u32, u64, (torch.uint8,)


class Engine:
    """One hcrc context (device tables, stream, pinned staging) per GPU."""

    def __init__(self, device: int = 0):
        self._lib = _lib.load()
        ctx = ctypes.c_void_p()
        check(self._lib.hcrc_ctx_create(device, ctypes.byref(ctx)), f"hcrc_ctx_create({device})")
        self._ctx = ctx
        self.device = device

    def close(self) -> None:
        if self._ctx:
            self._lib.hcrc_ctx_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def stream(self) -> int:
        return int(self._lib.hcrc_ctx_stream(self._ctx) or 0)

    # -- host memory ------------------------------------------------------
    def batch(self, base, offsets, lengths, inits=None, mask_output: bool = False) -> np.ndarray:
        """Synchronous batch over host memory (pinned staging, H2D, kernel, D2H)."""
        base = _as_bytes(base)
        off = np.ascontiguousarray(offsets, dtype=np.uint64)
        ln = np.ascontiguousarray(lengths, dtype=np.uint32)
        ini = None if inits is None else np.ascontiguousarray(inits, dtype=np.uint32)
        out = np.empty(off.size, dtype=np.uint32)
        flags = HCRC_MASK_OUTPUT if mask_output else 0
        check(self._lib.hcrc_batch(self._ctx, _ptr(base), _ptr(off), _ptr(ln), _ptr(ini),
                                   _ptr(out), off.size, flags), "hcrc_batch")
        return out

    # -- device memory (torch tensors on this device) ----------------------
    @staticmethod
    def _stream_of(stream) -> int:
        if stream is None:
            import torch
            return int(torch.cuda.current_stream().cuda_stream)
        if hasattr(stream, "cuda_stream"):  # a torch.cuda.Stream
            return int(stream.cuda_stream)
        return int(stream)

    def _device(self):
        import torch
        return torch.device("cuda", self.device)

    def _check_spans(self, base_t, offsets_t, lengths_t, inits_t, check_bounds: bool,
                     extra: int = 0, stream=None) -> int:
        u32, u64, _ = _dtypes()
        dev = self._device()
        _check_tensor(base_t, "base", dev, None)
        _check_tensor(offsets_t, "offsets", dev, u64)
        n = int(offsets_t.numel())
        _check_tensor(lengths_t, "lengths", dev, u32, n)
        _check_tensor(inits_t, "inits", dev, u32, n)
        if check_bounds and n:
            nbytes = base_t.numel() * base_t.element_size()
            self.check_spans(nbytes, offsets_t, lengths_t, extra, stream)
        return n

    def batch_device(self, base_t, offsets_t, lengths_t, inits_t=None, out_t=None,
                     mask_output: bool = False, stream=None, split_small: bool = False,
                     check_bounds: bool = False, split_long: bool = False,
                     balance: bool = False, packed: bool = False):
        """Asynchronous batch on device tensors; returns the uint32 out tensor
        (int32 storage).  Enqueued on ``stream`` (default: torch's current).
        ``split_small``: HCRC_SPLIT_SMALL (the size classes); ``split_long``:
        HCRC_SPLIT_LONG (spans of >= 128 KiB in 16 KiB parts on many waves;
        batches of at most 16 spans take it by themselves); ``balance``:
        HCRC_BALANCE (byte-balanced workgroup ranges for mixed sizes); ``packed``:
        HCRC_PACKED (an SST-packed batch -- sorted, no overlap, gaps < 4 KiB --
        read as one byte stream; checked on the device, a batch that is not
        packed runs the default pipeline).  Offsets are
        int64, lengths / inits / out 32-bit, all contiguous on this engine's
        device; ``check_bounds`` also checks every span against base (a
        device kernel and a sync, hcrc_check_spans)."""
        import torch
        n = self._check_spans(base_t, offsets_t, lengths_t, inits_t, check_bounds, 0, stream)
        if out_t is None:
            out_t = torch.empty(n, dtype=torch.int32, device=base_t.device)
        _check_tensor(out_t, "out", self._device(), _dtypes()[0], n)
        flags = HCRC_DEVICE_PTRS | (HCRC_MASK_OUTPUT if mask_output else 0)
        if split_small:
            flags |= HCRC_SPLIT_SMALL
        if split_long:
            flags |= HCRC_SPLIT_LONG
        if balance:
            flags |= HCRC_BALANCE
        if packed:
            flags |= HCRC_PACKED
        check(self._lib.hcrc_batch_async(self._ctx, _ptr(base_t), _ptr(offsets_t), _ptr(lengths_t),
                                         _ptr(inits_t), _ptr(out_t), n, flags,
                                         self._stream_of(stream)), "hcrc_batch_async")
        return out_t

    def batch_strided_device(self, base_t, stride: int, length: int, count: int, init: int = 0,
                             out_t=None, mask_output: bool = False, stream=None):
        import torch
        _check_tensor(base_t, "base", self._device(), None)
        if count and (count - 1) * stride + length > base_t.numel() * base_t.element_size():
            raise ValueError("the strided blocks run past base")
        if out_t is None:
            out_t = torch.empty(count, dtype=torch.int32, device=base_t.device)
        _check_tensor(out_t, "out", self._device(), _dtypes()[0], count)
        flags = HCRC_DEVICE_PTRS | (HCRC_MASK_OUTPUT if mask_output else 0)
        check(self._lib.hcrc_batch_strided_async(self._ctx, _ptr(base_t), stride, length,
                                                 init & 0xFFFFFFFF, _ptr(out_t), count, flags,
                                                 self._stream_of(stream)),
              "hcrc_batch_strided_async")
        return out_t

    def check_spans(self, base_bytes: int, offsets_t, lengths_t, extra: int = 0,
                    stream=None) -> None:
        """hcrc_check_spans_async: every span [offsets[i], +lengths[i] + extra)
        must lie in [0, base_bytes); raises IndexError naming the first that
        does not.  A device kernel on ``stream`` (default: torch's current,
        so it sees descriptors written there), then a sync of it."""
        import torch
        u32, u64, _ = _dtypes()
        _check_tensor(offsets_t, "offsets", self._device(), u64)
        n = int(offsets_t.numel())
        _check_tensor(lengths_t, "lengths", self._device(), u32, n)
        res = torch.empty(2, dtype=torch.int64, device=self._device())
        check(self._lib.hcrc_check_spans_async(self._ctx, int(base_bytes), _ptr(offsets_t),
                                               _ptr(lengths_t), int(extra), n, _ptr(res),
                                               self._stream_of(stream)),
              "hcrc_check_spans_async")
        self.sync(self._stream_of(stream))
        bad, first = (int(x) for x in res.cpu().numpy().view(np.uint64))
        if bad:
            raise IndexError(f"{bad} span(s) outside base ({base_bytes} bytes), first: {first}")

    def verify_device(self, base_t, offsets_t, lengths_t, status_t=None, stream=None,
                      split_small: bool = False, check_bounds: bool = False):
        """ReadBlock's check on device blocks: status[i] = 1 iff the stored
        masked crc at byte n+1 matches Value(block, n+1).  ``split_small``:
        HCRC_SPLIT_SMALL (small blocks and table-block remainders on the
        small-span kernel)."""
        import torch
        n = self._check_spans(base_t, offsets_t, lengths_t, None, check_bounds, 5, stream)
        if status_t is None:
            status_t = torch.zeros(n, dtype=torch.uint8, device=base_t.device)
        _check_tensor(status_t, "status", self._device(), _dtypes()[2], n)
        check(self._lib.hcrc_verify_async_ex(self._ctx, _ptr(base_t), _ptr(offsets_t),
                                             _ptr(lengths_t), _ptr(status_t), n,
                                             HCRC_SPLIT_SMALL if split_small else 0,
                                             self._stream_of(stream)),
              "hcrc_verify_async_ex")
        return status_t

    def readstream_device(self, base_t, stride: int, length: int, count: int, out_t=None,
                          stream=None):
        import torch
        if out_t is None:
            out_t = torch.empty(count, dtype=torch.int32, device=base_t.device)
        check(self._lib.hcrc_readstream_async(self._ctx, _ptr(base_t), stride, length,
                                              _ptr(out_t), count, self._stream_of(stream)),
              "hcrc_readstream_async")
        return out_t

    def dma_ceiling_device(self, base_t, stride: int, count: int, out_t=None, stream=None):
        """The spans kernel's memory side alone on `count` aligned 4 KiB blocks
        at `stride` (hcrc_dma_ceiling_async): the same-box ceiling of the
        roofline.  out[i] = XOR of the first 64 bytes of block i."""
        import torch
        nbytes = int(base_t.numel()) * base_t.element_size()
        if count and (count - 1) * stride + 4096 > nbytes:
            raise ValueError("dma_ceiling_device: the blocks run past the buffer")
        if out_t is None:
            out_t = torch.empty(count, dtype=torch.int32, device=base_t.device)
        if int(out_t.numel()) < count:
            raise ValueError("dma_ceiling_device: out is shorter than count")
        check(self._lib.hcrc_dma_ceiling_async(self._ctx, _ptr(base_t), stride, 4096,
                                               _ptr(out_t), count, self._stream_of(stream)),
              "hcrc_dma_ceiling_async")
        return out_t

    def fill_splitmix64_device(self, dst_t, seed: int, first_word: int = 0, stream=None):
        """Fill a device tensor with the seeded splitmix64 stream."""
        nbytes = int(dst_t.numel()) * dst_t.element_size()
        check(self._lib.hcrc_fill_splitmix64_async(self._ctx, _ptr(dst_t), nbytes, seed,
                                                   first_word, self._stream_of(stream)),
              "hcrc_fill_splitmix64_async")
        return dst_t

    def sync(self, stream=None) -> None:
        """hcrc_sync on ``stream`` (default: torch's current stream, as the
        async entry points): waits for it, then raises HCRC_ERR_KERNEL if one
        of this context's launches on that stream reported an in-kernel
        fault since the stream's last check."""
        check(self._lib.hcrc_sync(self._ctx, self._stream_of(stream)), "hcrc_sync")

    def stream_forget(self, stream) -> None:
        """hcrc_stream_forget: release this context's fault word and packed
        scratch for ``stream`` once its launches are complete, before the
        stream is destroyed; raises HCRC_ERR_KERNEL if its word held an
        unread fault."""
        check(self._lib.hcrc_stream_forget(self._ctx, self._stream_of(stream)),
              "hcrc_stream_forget")


def batch_multi(devices: Sequence[int], base, offsets, lengths, inits=None,
                mask_output: bool = False, shard_status: bool = False):
    """Host batch sharded by bytes over several GPUs (no collective).  With
    ``shard_status`` returns (out, per-shard return codes) without raising;
    a device may be listed more than once."""
    lib = _lib.load()
    base = _as_bytes(base)
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    ln = np.ascontiguousarray(lengths, dtype=np.uint32)
    ini = None if inits is None else np.ascontiguousarray(inits, dtype=np.uint32)
    out = np.empty(off.size, dtype=np.uint32)
    devs = (ctypes.c_int * len(devices))(*devices)
    rcs = (ctypes.c_int * len(devices))()
    flags = HCRC_MASK_OUTPUT if mask_output else 0
    rc = lib.hcrc_batch_multi_ex(devs, len(devices), _ptr(base), _ptr(off), _ptr(ln), _ptr(ini),
                                 _ptr(out), off.size, flags, rcs)
    if shard_status:
        return out, list(rcs)
    check(rc, "hcrc_batch_multi_ex")
    return out


__all__ = [
    "MASK_DELTA", "extend", "value", "mask", "unmask", "is_fast_crc32_supported",
    "cpu_batch", "device_count", "Engine", "batch_multi", "HcrcError",
]
