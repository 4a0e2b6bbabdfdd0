"""Synthetic CIFAR-shaped data resident in HBM (replaces main.py:65-91 CIFAR10 + DataLoaders).

Spec (DESIGN.md "Data spec"), shared with the test oracle but implemented independently here:
  * pool: POOL_SIZE uint8 images 3x32x32, label j % 10, image = clip(prototype[label] + noise)
    with prototypes ~ RandomState(seed).randint(0,256) and noise ~ RandomState(seed+1)
    .randint(-48, 49);
  * non-IID split (main.py:77-80): the first n-1 datasets are classes {0,2,..,8}, the last {1,9};
    the dataset of worker-step (t, i) is k = np.random.randint(0, n) from the seeded global
    numpy stream (main.py:138), drawn for every worker every epoch;
  * 128 samples with replacement (main.py:85 RandomSampler(replacement=True)): slot j takes
    list_k[philox(seed, t, i, SITE_DATA, j) % len(list_k)] -- drawn on the GPU;
  * ToTensor + Normalize(0.5, 0.5) (main.py:65-67) as a 256-entry fp32 table.
"""
from __future__ import annotations

import numpy as np
import torch

POOL_SIZE = 50000
TEST_SIZE = 10000
CLASSES_A = (0, 2, 3, 4, 5, 6, 7, 8)
CLASSES_B = (1, 9)


def make_pool(seed=0, size=POOL_SIZE, noise_seed=None):
    rs = np.random.RandomState(seed)
    proto = rs.randint(0, 256, size=(10, 3, 32, 32)).astype(np.int16)
    labels = (np.arange(size) % 10).astype(np.int64)
    noise_rs = np.random.RandomState(seed + 1 if noise_seed is None else noise_seed)
    imgs = np.empty((size, 3, 32, 32), np.uint8)
    for s in range(0, size, 5000):
        e = min(size, s + 5000)
        noise = noise_rs.randint(-48, 49, size=(e - s, 3, 32, 32)).astype(np.int16)
        imgs[s:e] = np.clip(proto[labels[s:e]] + noise, 0, 255).astype(np.uint8)
    return imgs, labels


def make_test_pool(seed=0, size=TEST_SIZE):
    """The test split (main.py:72-73 CIFAR10(train=False), 10,000 images, 1,000 per class):
    the training pool's class prototypes with an independent noise stream (seed + 2)."""
    return make_pool(seed, size, noise_seed=seed + 2)


def load_cifar10_bin(data_dir):
    """Real CIFAR-10 from a local copy of the binary distribution (cifar-10-batches-bin:
    data_batch_1..5.bin, test_batch.bin; records of 1 label byte + 3072 pixel bytes, R/G/B
    planes of 32x32) -- the same NCHW u8 layout as the synthetic pool.  Returns
    ((train_imgs, train_labels), (test_imgs, test_labels)).  No network access, no pickle."""
    import os

    def read(names):
        raw = b"".join(open(os.path.join(data_dir, n), "rb").read() for n in names)
        a = np.frombuffer(raw, np.uint8)
        if a.size % 3073:
            raise ValueError(f"{data_dir}: CIFAR-10 binary records are 3073 bytes")
        a = a.reshape(-1, 3073)
        return np.ascontiguousarray(a[:, 1:].reshape(-1, 3, 32, 32)), a[:, 0].astype(np.int64)

    train = read([f"data_batch_{i}.bin" for i in range(1, 6)])
    test = read(["test_batch.bin"])
    return train, test


def normalize_lut():
    u = np.arange(256, dtype=np.float32)
    return ((u / np.float32(255.0)) - np.float32(0.5)) / np.float32(0.5)


class DevicePool:
    """The pool, labels, class lists and normalisation table uploaded once to HBM (the train
    split; a test split uses the same class with pool=make_test_pool(seed))."""

    def __init__(self, device, seed=0, pool=None):
        imgs, labels = pool if pool is not None else make_pool(seed)
        self.device = device
        self.imgs = torch.from_numpy(np.ascontiguousarray(imgs)).to(device)
        self.labels = torch.from_numpy(labels.astype(np.int32)).to(device)
        a = np.where(np.isin(labels, CLASSES_A))[0].astype(np.int32)
        b = np.where(np.isin(labels, CLASSES_B))[0].astype(np.int32)
        self.list_a = torch.from_numpy(a).to(device)
        self.list_b = torch.from_numpy(b).to(device)
        self.lut = torch.from_numpy(normalize_lut()).to(device)
