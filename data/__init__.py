"""
Data loading (L5), API-compatible with the reference ``data/__init__.py``
(reference: data/__init__.py:1-38): ``load_data_from_args(split, data_dir,
batch_size, deterministic=False, loop=True, num_loader_proc=1)`` returns an
infinite generator of dict batches.

Additions (keyword-only, all optional): which dataset to build, sequence
shape, per-rank sharding (``shard=True`` gives each rank a disjoint slice -
the reference shuffles the whole dataset on every rank, SURVEY Q10, which
stays the default), and pinned host memory so the per-micro-batch H2D copy is
asynchronous.
"""
import torch

from .dataset import (CustomDataset, Seq2SeqJsonlDataset, SyntheticLMDataset,
                      SyntheticSeq2SeqDataset)


def _identity_collate(batch):
    return batch


def make_dataset(split, data_dir, *, dataset="synthetic", seq_len=128, vocab_size=30522, seed=0,
                 model="diffuseq", n_samples=None):
    if dataset in ("synthetic", "dataset") or dataset.startswith("synthetic"):
        n = n_samples or (1 << 20 if split == "train" else 1 << 14)
        if model == "gpt2":
            return SyntheticLMDataset(n, seq_len, vocab_size, seed, split)
        return SyntheticSeq2SeqDataset(n, seq_len, vocab_size, seed, split)
    return Seq2SeqJsonlDataset(data_dir, split, seq_len, vocab_size)


def load_data_from_args(
        split,
        data_dir,
        batch_size,
        deterministic=False,
        loop=True,
        num_loader_proc=1,
        *,
        dataset="synthetic",
        seq_len=128,
        vocab_size=30522,
        seed=0,
        model="diffuseq",
        shard=False,
        rank=0,
        world_size=1,
        pin_memory=None,
):
    from torch.utils.data import DataLoader
    from torch.utils.data.distributed import DistributedSampler

    data = make_dataset(split, data_dir, dataset=dataset, seq_len=seq_len, vocab_size=vocab_size,
                        seed=seed, model=model)
    sampler = None
    shuffle = not deterministic
    if shard and world_size > 1:
        sampler = DistributedSampler(data, num_replicas=world_size, rank=rank, shuffle=shuffle,
                                     seed=seed, drop_last=True)
        shuffle = False
    batched = hasattr(data, "__getitems__")
    pin = torch.cuda.is_available() if pin_memory is None else pin_memory
    collate = _identity_collate if batched else None  # pinning happens in the main process
    loader = DataLoader(
        data,
        batch_size=batch_size,
        shuffle=shuffle,
        sampler=sampler,
        num_workers=num_loader_proc,
        persistent_workers=num_loader_proc > 0,
        collate_fn=collate,
        pin_memory=pin,
        drop_last=True,
    )
    if loop:
        return infinite_loader_from_iterable(loader, sampler)
    return loader


def infinite_loader_from_object(obj):
    import copy
    while True:
        yield copy.deepcopy(obj)


def infinite_loader_from_iterable(iterable, sampler=None):
    epoch = 0
    while True:
        if sampler is not None and hasattr(sampler, "set_epoch"):
            sampler.set_epoch(epoch)
        yield from iterable
        epoch += 1


__all__ = ["load_data_from_args", "infinite_loader_from_object", "infinite_loader_from_iterable",
           "make_dataset", "CustomDataset", "SyntheticSeq2SeqDataset", "SyntheticLMDataset",
           "Seq2SeqJsonlDataset"]
