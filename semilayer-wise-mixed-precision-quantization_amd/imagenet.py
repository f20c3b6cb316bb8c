"""Drop-in for the reference's ``imagenet`` module (imagenet.py:1-40): exposes ``val_loader``.

The reference builds ``ImageFolder('./hogehoge/val')`` with Resize(256)/CenterCrop(224)/
Normalize and a DataLoader(batch_size=256, num_workers=16, pin_memory=True). That needs
torchvision and the ImageNet files. Like the reference, a missing dataset is an error: a search
run on random images would produce meaningless accuracies and KL orderings. A deterministic
synthetic stand-in of the same shape (N(0,1) 224x224 images, comparable to normalized ImageNet,
with seeded labels; ``SMPQ_SYNTH_IMAGES`` images, default 1024, in batches of ``SMPQ_BATCH``,
default 256) is served only on explicit opt-in, ``SMPQ_SYNTHETIC=1`` (the build and GPU boxes
have neither torchvision nor ImageNet), and announces itself on stderr.
"""
import os
import sys

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


if os.environ.get("SMPQ_SYNTHETIC", "0") == "1":
    print("smpq imagenet: SMPQ_SYNTHETIC=1 -> synthetic N(0,1) val_loader (%s images), not ImageNet"
          % os.environ.get("SMPQ_SYNTH_IMAGES", "1024"), file=sys.stderr)
    val_loader = SyntheticImageNet(int(os.environ.get("SMPQ_SYNTH_IMAGES", "1024")), BATCH)
else:
    val_loader = _real_loader()  # raises like the reference when torchvision / the dataset is absent
