"""Datasets for config-driven training (`mlcomp/contrib/dataset/{classify,segment,video}.py`).

* ``ImageDataset`` - images listed by a ``fold.csv`` (``image``, optional ``label``,
  ``fold``; train = fold != k, test = fold == k) or a whole folder; tiff / npy / any PIL
  format; albumentations-style ``transforms(image=..., mask=...)``; meta columns;
  ``max_count`` (int, or per-class list keeping the class ratio).
* ``ImageWithMaskDataset`` - adds masks (one-hot ``targets`` [C,H,W], or class ids with
  ``targets_encoded``), ``crop_positive`` (random crops centred on a positive region with
  probability 1-p), per-class ``empty_*`` flags.
* ``VideoDataset`` - clips of ``clip_length_in_frames`` frames from frame folders or
  ``.npy`` [T,H,W,C] arrays (no video decoder in this stack), clip index metadata cached
  as JSON, the same random transform applied to every frame of a clip.

Items are dicts with ``features`` (float32 CHW / CTHW) and ``targets``.  Images are read
with PIL (OpenCV is not part of this stack); connected regions for ``crop_positive`` use
scipy.ndimage.
"""
from __future__ import annotations

import ast
import json
import os
import random
from collections import defaultdict
from numbers import Number
from os.path import join
from typing import Callable, Dict, Optional

import numpy as np
from torch.utils.data import Dataset

from mlcomp_amd.train.data import register_dataset


def read_image_file(path: str, gray_scale: bool = False) -> np.ndarray:
    if not os.path.exists(path):
        raise FileNotFoundError(f'Image at path {path} does not exist')
    if path.endswith('.npy'):
        return np.load(path)
    from PIL import Image
    with Image.open(path) as im:
        if gray_scale:
            return np.asarray(im.convert('L'), dtype=np.uint8)
        if path.endswith(('.tif', '.tiff')) and im.mode not in ('RGB', 'L', 'P'):
            return np.asarray(im)
        return np.asarray(im.convert('RGB'))


def _load_rows(folder: str, fold_csv: Optional[str], fold: Optional[int], is_test: bool, col: str):
    import pandas as pd
    if fold_csv:
        df = pd.read_csv(fold_csv)
        if fold is not None:
            df = df[df['fold'] == fold] if is_test else df[df['fold'] != fold]
    else:
        df = pd.DataFrame({col: sorted(os.listdir(folder))})
    return df.to_dict(orient='records')


def _apply_max_count(rows, max_count):
    if max_count is None:
        return rows
    if isinstance(max_count, Number):
        return rows[:int(max_count)]
    by = defaultdict(list)
    for r in rows:
        by[r['label']].append(r)
    k_min = int(np.argmin(max_count))
    base = len(by[k_min])
    out = []
    for k in sorted(by):
        out += by[k][:int(base * max_count[k] / max_count[k_min])]
    return out


@register_dataset('image')
class ImageDataset(Dataset):
    def __init__(self, *, img_folder: str, fold_csv: str = None, fold: int = None, is_test: bool = False,
                 gray_scale: bool = False, num_classes=2, max_count=None, meta_cols=(), transforms=None,
                 postprocess_func: Callable[[Dict], Dict] = None, include_image_orig=False, **_):
        self.img_folder = img_folder
        self.data = _apply_max_count(_load_rows(img_folder, fold_csv, fold, is_test, 'image'), max_count)
        for row in self.data:
            self.preprocess_row(row)
        self.transforms = transforms
        self.gray_scale = gray_scale
        self.num_classes = num_classes
        self.meta_cols = list(meta_cols)
        self.postprocess_func = postprocess_func
        self.include_image_orig = include_image_orig

    read_image_file = staticmethod(read_image_file)

    def preprocess_row(self, row: dict):
        row['image'] = join(self.img_folder, row['image'])

    def __len__(self):
        return len(self.data)

    def _get_item_before_transform(self, row: dict, item: dict):
        pass

    def _get_item_after_transform(self, row: dict, transformed: dict, res: dict):
        if 'label' in row:
            t = ast.literal_eval(str(row['label']))
            res['targets'] = np.array(t, dtype=np.float32) if isinstance(t, list) else t

    def __getitem__(self, index):
        row = self.data[index]
        image = self.read_image_file(row['image'], self.gray_scale)
        item = {'image': image}
        self._get_item_before_transform(row, item)
        if self.transforms:
            item = self.transforms(**item)
        img = np.asarray(item['image'])
        if img.ndim == 2:
            img = img[None]
        elif img.ndim == 3 and img.shape[-1] in (1, 3, 4) and img.shape[0] not in (1, 3, 4):
            img = np.transpose(img, (2, 0, 1))    # HWC -> CHW unless the transform already did it
        res = {'features': img.astype(np.float32), 'image_file': row['image']}
        if self.include_image_orig:
            res['image'] = image
        for c in self.meta_cols:
            res[c] = row[c]
        self._get_item_after_transform(row, item, res)
        if self.postprocess_func:
            res = self.postprocess_func(res)
        return res


def _positive_box(mask: np.ndarray):
    """Bounding box (y, x, h, w) of a random connected positive region."""
    from scipy import ndimage
    lab, n = ndimage.label(mask > 0)
    k = np.random.randint(1, n + 1)
    sl = ndimage.find_objects(lab)[k - 1]
    return sl[0].start, sl[1].start, sl[0].stop - sl[0].start, sl[1].stop - sl[1].start


@register_dataset('image_with_mask')
class ImageWithMaskDataset(ImageDataset):
    def __init__(self, *, mask_folder: str, crop_positive=None, encode=True, include_binary=False, **kwargs):
        assert mask_folder, 'Mask folder is required'
        self.mask_folder = mask_folder
        self.crop_positive = crop_positive
        self.encode = encode
        self.include_binary = include_binary
        if not encode and kwargs.get('num_classes', 1) > 1:
            kwargs['num_classes'] += 1
        super().__init__(**kwargs)

    def preprocess_row(self, row: dict):
        row['image'] = join(self.img_folder, row['image'])
        if 'mask' in row:
            row['mask'] = join(self.mask_folder, row['mask'])

    def _get_item_before_transform(self, row: dict, item: dict):
        if 'mask' in row and self.mask_folder:
            item['mask'] = self.read_image_file(row['mask'], True)
            self._process_crop_positive(item)

    def _get_item_after_transform(self, row: dict, transformed: dict, res: dict):
        if 'mask' not in transformed:
            return
        mask = np.asarray(transformed['mask']).astype(np.int64)
        if mask.ndim == 2:
            enc = np.zeros((self.num_classes, *mask.shape), dtype=np.float32)
            if self.num_classes == 1:
                mask = (mask >= 1).astype(np.int64)
            for i in range(1, self.num_classes + 1):
                enc[i - 1] = mask == i
            if self.encode:
                mask = enc
            else:
                res['targets_encoded'] = enc
        res['targets'] = mask.astype(np.float32)
        if self.include_binary:
            for i, c in enumerate(np.atleast_3d(mask) if mask.ndim == 3 else [mask]):
                res[f'empty_{i}'] = int(c.sum() == 0)
            res['empty_all'] = int(mask.sum() == 0)

    def _process_crop_positive(self, item: dict):
        if not self.crop_positive:
            return
        mask = item['mask']
        H, W = mask.shape[:2]
        ch, cw, p = self.crop_positive
        ch = np.random.randint(*ch) if isinstance(ch, (tuple, list)) else ch
        cw = np.random.randint(*cw) if isinstance(cw, (tuple, list)) else cw
        if mask.sum() == 0 or np.random.uniform() < p:
            y0, y1, x0, x1 = 0, H - ch, 0, W - cw
        else:
            by, bx, bh, bw = _positive_box(mask)
            y0, y1 = by + bh // 2 - ch, by + bh // 2
            x0, x1 = bx + bw // 2 - cw, bx + bw // 2
        y0, x0 = max(0, y0), max(0, x0)
        y1, x1 = max(y0, min(y1, H - ch)), max(x0, min(x1, W - cw))
        y, x = np.random.randint(y0, y1 + 1), np.random.randint(x0, x1 + 1)
        item['image'] = item['image'][y:y + ch, x:x + cw]
        item['mask'] = mask[y:y + ch, x:x + cw]


class VideoClipsFolder:
    """Clip index over frame folders (or ``.npy`` videos): every
    ``frames_between_clips``-th window of ``clip_length_in_frames`` frames."""

    def __init__(self, video_paths, clip_length_in_frames: int, frames_between_clips: int,
                 _precomputed_metadata: dict = None):
        self.video_paths = list(video_paths)
        self.clip_length_in_frames = clip_length_in_frames
        self.frames_between_clips = frames_between_clips
        if _precomputed_metadata is not None:
            self.metadata = _precomputed_metadata
            self.clips = self.metadata['clips']
            self.cumulative_sizes = self.metadata['cumulative_sizes']
            self.video_paths = self.metadata['video_paths']
        else:
            self.compute_clips()

    @staticmethod
    def num_frames(path: str) -> int:
        if path.endswith('.npy'):
            return int(np.load(path, mmap_mode='r').shape[0])
        return len(os.listdir(path))

    def compute_clips(self):
        self.clips, self.cumulative_sizes = [], []
        total = 0
        for vi, path in enumerate(self.video_paths):
            n = self.num_frames(path)
            assert n >= self.clip_length_in_frames, f'{path} has only {n} frames'
            for i in range(0, n - self.clip_length_in_frames + 1, self.frames_between_clips):
                self.clips.append({'video_index': vi, 'min_index': i, 'max_index': i + self.clip_length_in_frames})
                total += 1
            self.cumulative_sizes.append(total)
        self.metadata = {'clips': self.clips, 'cumulative_sizes': self.cumulative_sizes,
                         'video_paths': self.video_paths}

    def get_clip(self, index: int):
        c = self.clips[index]
        path = self.video_paths[c['video_index']]
        if path.endswith('.npy'):
            frames = list(np.load(path, mmap_mode='r')[c['min_index']:c['max_index']])
        else:
            files = sorted(os.listdir(path))[c['min_index']:c['max_index']]
            frames = [read_image_file(join(path, f)) for f in files]
        return frames, None, None, c['video_index']


@register_dataset('video')
class VideoDataset(Dataset):
    def __init__(self, *, video_folder: str, fold_csv: str = None, fold: int = None, is_test: bool = False,
                 clip_length_in_frames: int = 1, frames_between_clips: int = 1, num_classes=2, max_count=None,
                 transforms=None, postprocess_func: Callable[[Dict], Dict] = None, clips_per_video: int = 1,
                 metadata_path: str = None, seed: int = 0, **_):
        self.video_folder = video_folder
        rows = _load_rows(video_folder, fold_csv, fold, is_test, 'video')
        random.Random(seed).shuffle(rows)
        self.data = _apply_max_count(rows, max_count)
        for row in self.data:
            row['video'] = join(video_folder, row['video'])
        self.transforms = transforms
        self.num_classes = num_classes
        self.postprocess_func = postprocess_func
        self.clips_per_video = clips_per_video
        self.metadata_path = metadata_path
        self.video_paths = [r['video'] for r in self.data]
        self.clips = self._create_clips(clip_length_in_frames, frames_between_clips)

    def _create_clips(self, length, between):
        meta = None
        if self.metadata_path and os.path.exists(self.metadata_path):
            with open(self.metadata_path) as f:
                meta = json.load(f)
            if meta.get('video_paths') != self.video_paths:
                meta = None
        clips = VideoClipsFolder(self.video_paths, length, between, meta)
        if meta is None and self.metadata_path:
            os.makedirs(os.path.dirname(self.metadata_path) or '.', exist_ok=True)
            with open(self.metadata_path, 'w') as f:
                json.dump(clips.metadata, f)
        return clips

    def __len__(self):
        return len(self.video_paths) * self.clips_per_video

    def __getitem__(self, index):
        vi = index // self.clips_per_video
        lo = self.clips.cumulative_sizes[vi - 1] if vi > 0 else 0
        ci = np.random.randint(lo, self.clips.cumulative_sizes[vi])
        frames, _, _, _ = self.clips.get_clip(ci)
        if self.transforms:
            seed = random.randint(0, 10 ** 6)
            out = []
            for f in frames:   # same random parameters on every frame
                random.seed(seed)
                np.random.seed(seed % (2 ** 32))
                out.append(self.transforms(image=np.asarray(f))['image'])
            frames = out
        clip = np.stack([np.asarray(f) for f in frames]).astype(np.float32)   # T,H,W,C
        res = {'features': np.transpose(clip, (3, 0, 1, 2))}                  # C,T,H,W
        row = self.data[vi]
        if 'label' in row:
            res['targets'] = ast.literal_eval(str(row['label']))
        if self.postprocess_func:
            res = self.postprocess_func(res)
        return res


__all__ = ['ImageDataset', 'ImageWithMaskDataset', 'VideoDataset', 'VideoClipsFolder', 'read_image_file']
