"""Drop-in for the reference's ``imagenet`` module (imagenet.py:1-40): exposes ``val_loader``.

The reference builds ``ImageFolder('./hogehoge/val')`` with Resize(256)/CenterCrop(224)/
Normalize and a DataLoader(batch_size=256, num_workers=16, pin_memory=True). That needs
torchvision and the ImageNet files; when either is missing (as on the build and GPU boxes)
this module serves a deterministic synthetic stand-in of the same shape: N(0,1) 224x224
images (comparable to normalized ImageNet) with seeded labels, ``SMPQ_SYNTH_IMAGES`` images
(default 1024) in batches of ``SMPQ_BATCH`` (default 256).
"""
import os

import torch

ROOT = os.environ.get("SMPQ_IMAGENET_ROOT", "./hogehoge")
BATCH = int(os.environ.get("SMPQ_BATCH", "256"))


class SyntheticImageNet:
    def __init__(self, n_images=1024, batch_size=256, seed=1, num_classes=1000):
        self.n_images, self.batch_size, self.seed, self.num_classes = n_images, batch_size, seed, num_classes

    def __len__(self):
        return (self.n_images + self.batch_size - 1) // self.batch_size

    def __iter__(self):
        g = torch.Generator().manual_seed(self.seed)
        for start in range(0, self.n_images, self.batch_size):
            b = min(self.batch_size, self.n_images - start)
            x = torch.randn(b, 3, 224, 224, generator=g)
            y = torch.randint(0, self.num_classes, (b,), generator=g)
            yield x, y


def _real_loader():
    import torchvision
    import torchvision.transforms as T
    tf = T.Compose([T.Resize(256), T.CenterCrop(224), T.ToTensor(),
                    T.Normalize(mean=[0.485, 0.456, 0.406], std=[0.229, 0.224, 0.225])])
    ds = torchvision.datasets.ImageFolder(os.path.join(ROOT, "val"), tf)
    return torch.utils.data.DataLoader(ds, batch_size=BATCH, shuffle=False, num_workers=16, pin_memory=True)


try:
    val_loader = _real_loader()
except Exception:  # torchvision or the dataset absent
    val_loader = SyntheticImageNet(int(os.environ.get("SMPQ_SYNTH_IMAGES", "1024")), BATCH)
