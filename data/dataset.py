"""
Datasets (L5).  The reference ships only a ``CustomDataset`` stub
(reference: data/dataset.py:1-15); here are the datasets its workloads need.

* :class:`SyntheticSeq2SeqDataset` - DiffuSeq-shaped samples from random tokens:
  ``[CLS] src [SEP] trg [SEP] pad...`` with ``input_mask`` 0 on the source and
  1 on target + padding (DiffuSeq's collate convention).  Deterministic per
  index (counter-based hashing) and *batched*: ``__getitems__`` builds a whole
  batch with a few vectorised numpy ops, so a 2048-sample batch costs
  ~1 ms of loader time instead of 2048 ``__getitem__`` calls.
* :class:`SyntheticLMDataset` - random token sequences for the GPT-2 path.
* :class:`Seq2SeqJsonlDataset` - DiffuSeq ``{"src": ..., "trg": ...}`` jsonl
  files tokenised offline (a local ``vocab.txt`` WordPiece vocab if present,
  else a deterministic hashing word tokenizer - there is no network).
* :class:`CustomDataset` - kept as the user extension point.
"""
import json
import os
import zlib

import numpy as np
import torch
from torch.utils.data import Dataset

CLS_ID, SEP_ID, PAD_ID = 101, 102, 0


def _splitmix64(x):
    x = (x + np.uint64(0x9E3779B97F4A7C15)) & np.uint64(0xFFFFFFFFFFFFFFFF)
    z = x
    z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & np.uint64(0xFFFFFFFFFFFFFFFF)
    z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & np.uint64(0xFFFFFFFFFFFFFFFF)
    return z ^ (z >> np.uint64(31))


class _BatchedDataset(Dataset):
    """Dataset whose ``__getitems__`` returns an already-collated dict batch."""

    def __getitem__(self, idx):
        b = self.__getitems__([idx])
        return {k: v[0] for k, v in b.items()}

    def __getitems__(self, idxs):
        raise NotImplementedError


class SyntheticSeq2SeqDataset(_BatchedDataset):
    def __init__(self, n_samples=1 << 20, seq_len=128, vocab_size=30522, seed=0, split="train"):
        self.n, self.L, self.V = int(n_samples), int(seq_len), int(vocab_size)
        self.seed = (int(seed) * 1000003 + zlib.crc32(split.encode())) & 0xFFFFFFFF

    def __len__(self):
        return self.n

    def __getitems__(self, idxs):
        idx = np.asarray(idxs, dtype=np.uint64)
        B, L = idx.shape[0], self.L
        base = (np.uint64(self.seed) << np.uint64(32)) ^ (idx << np.uint64(12))
        pos = np.arange(L + 2, dtype=np.uint64)
        h = _splitmix64(base[:, None] ^ pos[None, :])
        lo = max(4, L // 4)
        body = max(lo + 2, L - 2)
        src_len = (lo + (h[:, L] % np.uint64(max(1, L // 4))).astype(np.int64))
        trg_len = (1 + (h[:, L + 1] % np.uint64(max(1, body - src_len.max()))).astype(np.int64))
        trg_len = np.minimum(trg_len, L - 3 - src_len)
        t0 = 1000 if self.V > 2000 else 103  # skip [PAD]/[CLS]/[SEP]-range ids
        tok = (t0 + (h[:, :L] % np.uint64(self.V - t0))).astype(np.int64)
        j = np.arange(L)[None, :]
        s_end = 1 + src_len[:, None]
        t_end = s_end + 1 + trg_len[:, None]
        ids = np.where(j < t_end + 1, tok, PAD_ID)
        ids = np.where(j == 0, CLS_ID, ids)
        ids = np.where(j == s_end, SEP_ID, ids)
        ids = np.where(j == t_end, SEP_ID, ids)
        mask = (j > s_end).astype(np.int64)
        return {"input_ids": torch.from_numpy(ids), "input_mask": torch.from_numpy(mask)}


class SyntheticLMDataset(_BatchedDataset):
    def __init__(self, n_samples=1 << 20, seq_len=1024, vocab_size=50257, seed=0, split="train"):
        self.n, self.L, self.V = int(n_samples), int(seq_len), int(vocab_size)
        self.seed = (int(seed) * 1000003 + zlib.crc32(split.encode())) & 0xFFFFFFFF

    def __len__(self):
        return self.n

    def __getitems__(self, idxs):
        idx = np.asarray(idxs, dtype=np.uint64)
        base = (np.uint64(self.seed) << np.uint64(32)) ^ (idx << np.uint64(16))
        h = _splitmix64(base[:, None] ^ np.arange(self.L, dtype=np.uint64)[None, :])
        ids = (h % np.uint64(self.V)).astype(np.int64)
        t = torch.from_numpy(ids)
        return {"input_ids": t, "labels": t.clone()}


class _HashTokenizer:
    """Deterministic offline word tokenizer (used when no vocab.txt is on disk)."""

    def __init__(self, vocab_size):
        self.V = vocab_size

    def encode(self, text):
        return [1000 + zlib.crc32(w.lower().encode()) % (self.V - 1000) for w in text.split()]


def _load_tokenizer(data_dir, vocab_size):
    vocab = os.path.join(data_dir, "vocab.txt")
    if os.path.exists(vocab):
        try:
            from transformers import BertTokenizerFast
            tok = BertTokenizerFast(vocab_file=vocab)

            class _Wrap:
                def encode(self, text):
                    return tok.encode(text, add_special_tokens=False)
            return _Wrap()
        except Exception:  # noqa: BLE001
            pass
    return _HashTokenizer(vocab_size)


class Seq2SeqJsonlDataset(_BatchedDataset):
    """DiffuSeq-format ``{data_dir}/{split}.jsonl`` with ``src``/``trg`` fields."""

    def __init__(self, data_dir, split="train", seq_len=128, vocab_size=30522):
        path = os.path.join(data_dir, f"{split}.jsonl")
        if not os.path.exists(path) and split == "valid":
            path = os.path.join(data_dir, "test.jsonl")
        tok = _load_tokenizer(data_dir, vocab_size)
        ids, masks = [], []
        with open(path) as f:
            for line in f:
                line = line.strip()
                if not line:
                    continue
                rec = json.loads(line)
                src, trg = tok.encode(rec["src"]), tok.encode(rec["trg"])
                while len(src) + len(trg) > seq_len - 3:  # DiffuSeq truncation
                    if len(src) > len(trg):
                        src.pop()
                    elif len(trg) > 0:
                        trg.pop()
                    else:
                        break
                s = [CLS_ID] + src + [SEP_ID]
                t = trg + [SEP_ID]
                row = s + t
                m = [0] * len(s) + [1] * len(t)
                row += [PAD_ID] * (seq_len - len(row))
                m += [1] * (seq_len - len(m))
                ids.append(row[:seq_len])
                masks.append(m[:seq_len])
        self.ids = torch.tensor(ids, dtype=torch.long)
        self.mask = torch.tensor(masks, dtype=torch.long)

    def __len__(self):
        return self.ids.shape[0]

    def __getitems__(self, idxs):
        ix = torch.as_tensor(idxs, dtype=torch.long)
        return {"input_ids": self.ids[ix], "input_mask": self.mask[ix]}


class CustomDataset(Dataset):
    """User extension point (reference data/dataset.py:5-15)."""

    def __init__(self, *args, **kwargs):
        raise NotImplementedError

    def __getitem__(self, item):
        raise NotImplementedError

    def __len__(self):
        raise NotImplementedError
