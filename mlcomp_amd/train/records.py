"""Record files and the native input pipeline.

The reference trains from a PyTorch ``DataLoader`` over python datasets
(`mlcomp/contrib/dataset/classify.py:16-138`, driven by Catalyst).  On MI355X a step takes
~22 ms for 256 ImageNet images, so one node consumes ~92k images/s: the input pipeline is
split between the host and the GPU instead.

* ``.mlrec`` record file: fixed-size uint8 HWC images + int32 labels behind a 64-byte
  header (:func:`write_records`, :func:`pack_images`), memory-mapped by the C++ runtime
  (``csrc/runtime/records.cpp`` -> ``libmlcomp_runtime.so``).
* :class:`RecordLoader`: C++ worker threads copy the raw records of each batch into pinned
  ring slots and draw the per-sample augmentation (RandomResizedCrop box + flip, or the
  centre crop) from a counter-based RNG keyed by (seed, epoch, sample), so the stream is
  identical for any thread count.  Epochs are shuffled globally and sharded by rank.
  The uint8 batch crosses PCIe on a copy stream; one HIP kernel (``mlc_augment``,
  ``csrc/kernels/augment.hip``) crops, resizes, flips, normalises and writes the layout
  the model reads (the native ResNet stem's space-to-depth image, NHWC8 or NCHW fp32).
* :func:`augment_reference` is the same transform in PyTorch (CPU path, test oracle).
"""
from __future__ import annotations

import ctypes as C
import math
import weakref
import os
import struct
from typing import Iterable, Optional, Sequence, Tuple

import numpy as np
import torch

MAGIC = b'MLREC001'
HEADER = struct.Struct('<8s4I2Q24x')
LAYOUTS = {'s2d': 0, 'nhwc8': 1, 'nchw': 2}
IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


# ------------------------------------------------------------------------- files
def write_records(path: str, images: Iterable, labels: Optional[Iterable[int]] = None,
                  shape: Optional[Tuple[int, int, int]] = None) -> int:
    """Write ``images`` (uint8 HWC arrays of one shape, or one [N, H, W, C] array) and their
    int labels to ``path``; returns the record count.  Written to ``path + '.tmp'`` and
    renamed, so a reader never sees a partial file."""
    if isinstance(images, np.ndarray) and images.ndim == 4:
        shape = images.shape[1:]
    it = iter(images)
    first = None
    if shape is None:
        first = np.asarray(next(it), dtype=np.uint8)
        shape = first.shape
    H, W, Cc = (int(s) for s in shape)
    rec_bytes = H * W * Cc + 4
    labs = iter(labels) if labels is not None else None
    tmp = path + '.tmp'
    n = 0
    with open(tmp, 'wb') as f:
        f.write(HEADER.pack(MAGIC, H, W, Cc, 4, 0, rec_bytes))

        def put(img):
            nonlocal n
            a = np.ascontiguousarray(img, dtype=np.uint8)
            if a.shape != (H, W, Cc):
                raise ValueError(f'record {n}: shape {a.shape} != {(H, W, Cc)}')
            f.write(a.tobytes())
            f.write(struct.pack('<i', int(next(labs)) if labs is not None else 0))
            n += 1
        if first is not None:
            put(first)
        for img in it:
            put(img)
        f.seek(0)
        f.write(HEADER.pack(MAGIC, H, W, Cc, 4, n, rec_bytes))
    os.replace(tmp, path)
    return n


def pack_images(paths: Sequence[str], labels: Sequence[int], out: str, size: int = 256) -> int:
    """Decode image files (PIL), resize the shorter side to ``size``, centre-crop a
    ``size`` x ``size`` square and write them as a record file."""
    from PIL import Image

    def gen():
        for p in paths:
            im = Image.open(p).convert('RGB')
            w, h = im.size
            s = size / min(w, h)
            im = im.resize((max(size, round(w * s)), max(size, round(h * s))), Image.BILINEAR)
            w, h = im.size
            l, t = (w - size) // 2, (h - size) // 2
            yield np.asarray(im.crop((l, t, l + size, t + size)), dtype=np.uint8)
    return write_records(out, gen(), labels, shape=(size, size, 3))


class RecordFile:
    """numpy view of a record file (header checks, random access) - the python twin of the
    C++ reader, used by tests and tools."""

    def __init__(self, path: str):
        with open(path, 'rb') as f:
            magic, H, W, Cc, lb, n, rb = HEADER.unpack(f.read(HEADER.size))
        if magic != MAGIC or lb != 4 or rb != H * W * Cc + 4:
            raise ValueError(f'{path}: not an mlrec file')
        self.shape = (H, W, Cc)
        self.count = n
        self._m = np.memmap(path, dtype=np.uint8, mode='r', offset=HEADER.size, shape=(n, rb))

    def __len__(self):
        return self.count

    def image(self, i: int) -> np.ndarray:
        H, W, Cc = self.shape
        return np.asarray(self._m[i, :H * W * Cc]).reshape(H, W, Cc)

    def label(self, i: int) -> int:
        return int(np.asarray(self._m[i, -4:]).view('<i4')[0])


# ------------------------------------------------------------------------- runtime
_RT = None


def runtime():
    """ctypes handle of libmlcomp_runtime.so (built in-tree on first use)."""
    global _RT
    if _RT is not None:
        return _RT
    from mlcomp_amd.build import RUNTIME_LIB, build_runtime
    if not os.path.exists(RUNTIME_LIB):
        build_runtime()
    lib = C.CDLL(RUNTIME_LIB)
    vp, i32, i64, u64, f64 = C.c_void_p, C.c_int, C.c_int64, C.c_uint64, C.c_double
    sig = {
        'mlr_open': ([C.c_char_p], vp), 'mlr_close': ([vp], None), 'mlr_shape': ([vp, vp], None),
        'mlr_loader_create': ([vp, i32, i32, i32, i32, f64, f64, f64, f64, u64, i32, i32, i32, i32, i32, i32], vp),
        'mlr_loader_set_slot': ([vp, i32, vp, vp, vp], i32),
        'mlr_loader_start_epoch': ([vp, u64], i64),
        'mlr_loader_next': ([vp, vp], i32), 'mlr_loader_release': ([vp, i32], None),
        'mlr_loader_destroy': ([vp], None),
    }
    for name, (args, res) in sig.items():
        fn = getattr(lib, name)
        fn.argtypes, fn.restype = args, res
    _RT = lib
    return lib


def augment_reference(img: torch.Tensor, par: torch.Tensor, out_h: int, out_w: int, mean_istd: Sequence[float],
                      layout: str = 'nchw') -> torch.Tensor:
    """PyTorch twin of ``mlc_augment``: img uint8 [B, H, W, C], par int [B, 5]
    (y0, x0, h, w, flip) -> the normalised crops in ``layout``."""
    B, H, W, Cc = img.shape
    p = par.long()
    oy = torch.arange(out_h, dtype=torch.float32)
    ox = torch.arange(out_w, dtype=torch.float32)
    outs = []
    for b in range(B):
        y0, x0, h, w, flip = p[b].tolist()
        xs = (out_w - 1 - ox) if flip else ox
        fy = ((oy + 0.5) * (h / out_h) - 0.5).clamp(0, h - 1)
        fx = ((xs + 0.5) * (w / out_w) - 0.5).clamp(0, w - 1)
        iy0, ix0 = fy.floor().long(), fx.floor().long()
        iy1, ix1 = (iy0 + 1).clamp(max=h - 1), (ix0 + 1).clamp(max=w - 1)
        wy, wx = (fy - iy0)[:, None, None], (fx - ix0)[None, :, None]
        im = img[b].float()
        g = lambda yy, xx: im[y0 + yy][:, x0 + xx]  # noqa: E731
        top = g(iy0, ix0) + wx * (g(iy0, ix1) - g(iy0, ix0))
        bot = g(iy1, ix0) + wx * (g(iy1, ix1) - g(iy1, ix0))
        outs.append(top + wy * (bot - top))
    x = torch.stack(outs)                                   # [B, oh, ow, C] in 0..255
    mean = torch.tensor(mean_istd[:Cc])
    istd = torch.tensor(mean_istd[4:4 + Cc])
    x = (x - mean) * istd
    if layout == 'nchw':
        return x.permute(0, 3, 1, 2).contiguous()
    if layout == 'nhwc8':
        return torch.nn.functional.pad(x, (0, 8 - Cc)).to(torch.bfloat16)
    from mlcomp_amd.ops.functional import stem_s2d
    return stem_s2d(x.to(torch.bfloat16), 3)


class RecordLoader:
    """Batches of a record file: dicts {'features', 'targets'} on ``device``.

    ``train``: RandomResizedCrop(scale, ratio) + horizontal flip, reshuffled every epoch;
    otherwise the centre ``out_size`` crop in file order.  ``rank`` / ``world_size`` shard
    each epoch like a DistributedSampler (padding by wrap-around); ``drop_last`` (default:
    ``train``) drops a last partial batch, otherwise it is completed by wrapping.
    ``threads`` host workers, ``depth`` pinned ring slots (>= 3)."""

    def __init__(self, path: str, batch_size: int, out_size: int = 224, train: bool = True,
                 scale=(0.08, 1.0), ratio=(3 / 4, 4 / 3), seed: int = 0, rank: int = 0, world_size: int = 1,
                 shuffle: Optional[bool] = None, drop_last: Optional[bool] = None, threads: int = 8,
                 depth: int = 4, layout: str = 's2d', mean=IMAGENET_MEAN, std=IMAGENET_STD, device=None,
                 chunk: int = 16):
        self.path = path
        self.batch_size = int(batch_size)
        self.out_h = self.out_w = int(out_size)
        self.train = bool(train)
        self.layout = layout
        self.device = torch.device(device or ('cuda' if torch.cuda.is_available() else 'cpu'))
        self.epoch = 0
        self._explicit_epoch = False
        rt = runtime()
        self._rt = rt
        self._file = rt.mlr_open(path.encode())
        if not self._file:
            raise ValueError(f'{path}: cannot open record file')
        shp = (C.c_uint64 * 4)()
        rt.mlr_shape(self._file, shp)
        self.count, self.H, self.W, self.C = (int(v) for v in shp)
        if layout not in LAYOUTS or (layout == 's2d' and (self.C != 3 or self.out_h % 2)):
            raise ValueError(f'layout {layout!r} does not fit {self.C}-channel images of {out_size}')
        ms = [0.0] * 8
        for c in range(min(self.C, 4)):
            m, s = (mean[c], std[c]) if c < len(mean) else (0.0, 1.0)
            ms[c], ms[4 + c] = m * 255.0, 1.0 / (s * 255.0)
        self.mean_istd = ms
        shuffle = self.train if shuffle is None else shuffle
        drop_last = self.train if drop_last is None else drop_last
        per = math.ceil(self.count / world_size)
        self._per = per
        self._drop_last = bool(drop_last)
        self._live = None
        self._len = per // self.batch_size if drop_last else math.ceil(per / self.batch_size)
        self._loader = rt.mlr_loader_create(self._file, self.batch_size, self.out_h, self.out_w, int(self.train),
                                            float(scale[0]), float(scale[1]), float(ratio[0]), float(ratio[1]),
                                            int(seed), int(rank), int(world_size), int(shuffle), int(drop_last),
                                            int(threads), int(chunk))
        if not self._loader:
            raise ValueError('bad loader arguments')
        pin = self.device.type == 'cuda'
        B = self.batch_size
        self._slots = []
        for i in range(max(3, int(depth))):
            img = torch.empty(B, self.H, self.W, self.C, dtype=torch.uint8, pin_memory=pin)
            lab = torch.empty(B, dtype=torch.int64, pin_memory=pin)
            par = torch.empty(B, 5, dtype=torch.int32, pin_memory=pin)
            rt.mlr_loader_set_slot(self._loader, i, C.c_void_p(img.data_ptr()), C.c_void_p(lab.data_ptr()),
                                   C.c_void_p(par.data_ptr()))
            self._slots.append((img, lab, par))
        if self.device.type == 'cuda':
            self._copy_stream = torch.cuda.Stream(self.device)
            self._dev = [(torch.empty(B, self.H, self.W, self.C, dtype=torch.uint8, device=self.device),
                          torch.empty(B, 5, dtype=torch.int32, device=self.device)) for _ in range(2)]
            self._ms_dev = torch.tensor(ms, dtype=torch.float32, device=self.device)
            self._used = [None, None]   # event: the augment kernel that last read each staging buffer

    # the sampler-like API the runner calls
    @property
    def sampler(self):
        return self

    def set_epoch(self, epoch: int):
        self.epoch = int(epoch)
        self._explicit_epoch = True

    def __len__(self):
        return self._len

    @property
    def dataset(self):
        return range(self.count)

    def _out_shape(self, B):
        if self.layout == 's2d':
            return (B, (self.out_h + 6) // 2, (self.out_w + 6) // 2, 16), torch.bfloat16
        if self.layout == 'nhwc8':
            return (B, self.out_h, self.out_w, 8), torch.bfloat16
        return (B, self.C, self.out_h, self.out_w), torch.float32

    def _augment_gpu(self, k, slot):
        from mlcomp_amd.ops import _lib
        img, lab, par = slot
        dimg, dpar = self._dev[k % 2]
        cur = torch.cuda.current_stream(self.device)
        cs = self._copy_stream
        if self._used[k % 2] is not None:
            cs.wait_event(self._used[k % 2])
        with torch.cuda.stream(cs):
            dimg.copy_(img, non_blocking=True)
            dpar.copy_(par, non_blocking=True)
            dlab = lab.to(self.device, non_blocking=True)
            done = torch.cuda.Event()
            done.record(cs)
        cur.wait_event(done)
        dlab.record_stream(cur)
        shape, dt = self._out_shape(self.batch_size)
        out = torch.empty(shape, dtype=dt, device=self.device)
        _lib.call('mlc_augment', _lib.ptr(dimg), _lib.ptr(dpar), _lib.ptr(self._ms_dev), _lib.ptr(out),
                  self.batch_size, self.H, self.W, self.C, self.out_h, self.out_w, LAYOUTS[self.layout],
                  _lib.stream())
        used = torch.cuda.Event()
        used.record(cur)
        self._used[k % 2] = used
        return out, dlab, done

    def real_rows(self, k: int) -> int:
        """Samples of batch ``k`` that are not wrap-around padding.  Only the last batch of
        a ``drop_last=False`` epoch has padding: ``per - (len-1)*batch`` rows are real (the
        world-size padding of the shard stays, as DistributedSampler does it)."""
        if k < self._len - 1 or self._drop_last:
            return self.batch_size
        return self._per - (self._len - 1) * self.batch_size

    def __iter__(self):
        # an earlier iterator still alive holds an INUSE slot whose async H2D copy may be
        # pending: close it (its finally releases the slot) before the ring is reset
        prev = self._live() if self._live is not None else None
        if prev is not None:
            prev.close()
        gen = self._epoch_iter()
        self._live = weakref.ref(gen)
        return gen

    def _epoch_iter(self):
        rt = self._rt
        n = rt.mlr_loader_start_epoch(self._loader, self.epoch)
        if n < 0:
            raise RuntimeError('record loader: slots not registered')
        pending = None   # (slot index, copy-done event) of the previous batch
        bi = C.c_int64(0)
        try:
            for k in range(n):
                s = rt.mlr_loader_next(self._loader, C.byref(bi))
                if s < 0:
                    break
                slot = self._slots[s]
                if self.device.type == 'cuda':
                    x, y, done = self._augment_gpu(k, slot)
                else:
                    img, lab, par = slot
                    x = augment_reference(img, par, self.out_h, self.out_w, self.mean_istd, self.layout)
                    y = lab.clone()
                    done = None
                    rt.mlr_loader_release(self._loader, s)
                    s = -1
                if pending is not None:   # the previous slot's copy is long done: hand it back
                    ps, pev = pending
                    pev.synchronize()
                    rt.mlr_loader_release(self._loader, ps)
                pending = (s, done) if s >= 0 else None
                real = self.real_rows(k)
                if real < self.batch_size:   # drop the wrap-around rows of the last batch
                    x, y = x[:real], y[:real]
                yield {'features': x, 'targets': y}
        finally:
            if pending is not None:
                pending[1].synchronize()
                rt.mlr_loader_release(self._loader, pending[0])
            if not self._explicit_epoch:
                self.epoch += 1
            self._explicit_epoch = False

    def close(self):
        if getattr(self, '_loader', None):
            self._rt.mlr_loader_destroy(self._loader)
            self._loader = None
        if getattr(self, '_file', None):
            self._rt.mlr_close(self._file)
            self._file = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


__all__ = ['write_records', 'pack_images', 'RecordFile', 'RecordLoader', 'augment_reference', 'runtime']
