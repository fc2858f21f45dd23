"""Checkpoint-based image classification inference (`mlcomp/contrib/complex/infer.py:14-79`):
build ``Pretrained``/``Timm`` (or take ``model``), load ``model_state_dict`` from a
training checkpoint (``weights_only=True``), run files in batches with resize +
ImageNet normalisation (or custom ``transforms(image=...)``), return probabilities."""
from __future__ import annotations

from typing import List

import numpy as np
import torch


def _default_transform(size=224, mean=(0.485, 0.456, 0.406), std=(0.229, 0.224, 0.225)):
    from PIL import Image

    def t(image):
        im = Image.fromarray(image).resize((size, size), Image.BILINEAR)
        a = (np.asarray(im, dtype=np.float32) / 255.0 - np.array(mean, np.float32)) / np.array(std, np.float32)
        return {'image': np.transpose(a, (2, 0, 1))}
    return t


def infer(files: List[str], checkpoint: str, model=None, class_: str = 'Pretrained', variant: str = 'resnet34',
          activation: str = 'softmax', num_classes: int = 2, batch_size: int = 16, device: str = None,
          transforms=None) -> np.ndarray:
    assert activation in ('softmax', 'sigmoid', None)
    from mlcomp_amd.contrib.dataset import read_image_file
    from mlcomp_amd.models import build_model
    device = device or ('cuda' if torch.cuda.is_available() else 'cpu')
    if model is None:
        if class_ not in ('Pretrained', 'Timm'):
            raise ValueError('unknown model class')
        model = build_model(class_, variant=variant, num_classes=num_classes)
    transforms = transforms or _default_transform()
    ck = torch.load(checkpoint, map_location='cpu', weights_only=True)
    sd = ck.get('model_state_dict', ck)
    try:
        model.load_state_dict(sd)
    except RuntimeError:   # checkpoint of the bare backbone inside a Pretrained wrapper
        model.model.load_state_dict(sd)
    model = model.to(device).eval()
    preds = []
    for i in range(0, len(files), batch_size):
        batch = np.stack([transforms(image=read_image_file(f))['image'] for f in files[i:i + batch_size]])
        with torch.no_grad(), torch.autocast(device if device != 'cpu' else 'cpu', dtype=torch.bfloat16,
                                             enabled=device != 'cpu'):
            p = model(torch.from_numpy(batch).to(device)).float()
        if activation == 'softmax':
            p = torch.softmax(p, 1)
        elif activation == 'sigmoid':
            p = torch.sigmoid(p)
        preds.append(p.cpu().numpy())
    return np.concatenate(preds) if preds else np.zeros((0, num_classes))


__all__ = ['infer']
