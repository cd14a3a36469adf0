"""Copy-stream prefetch of training batches to the GPU (SURVEY K-2).

The reference moves each micro-batch with a blocking ``.to(dev)`` on the compute
stream inside the training loop (reference utils/trainer.py:210-213).  Here the whole
per-rank batch of the NEXT step is copied from pinned host memory on a dedicated
HIP stream while the current step computes; the consumer's stream waits on an event
recorded after the copy (no host synchronisation), and the device tensors are marked
as used by the consumer stream so the caching allocator never recycles them early.
Micro-batches are then device slices (views): no per-micro-batch transfers remain.
"""
import torch

from distributed_pipeline_amd.runtime.streams import plan_stream


class DevicePrefetcher:
    """Iterator over ``it`` yielding dict batches already resident on ``device``."""

    def __init__(self, it, device):
        self.it = iter(it)
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        self.stream = plan_stream(self.device, "copy") if self.cuda else None
        self._next = self._stage()

    def _stage(self):
        try:
            batch = next(self.it)
        except StopIteration:
            return None
        if not self.cuda or not isinstance(batch, dict):
            return batch, None
        with torch.cuda.stream(self.stream):
            out = {}
            for k, v in batch.items():
                if torch.is_tensor(v) and not v.is_cuda:
                    v = v.pin_memory().to(self.device, non_blocking=True)
                out[k] = v
            ev = torch.cuda.Event()
            ev.record(self.stream)
        return out, ev

    def __iter__(self):
        return self

    def __next__(self):
        if self._next is None:
            raise StopIteration
        batch, ev = self._next
        if ev is not None:
            cur = torch.cuda.current_stream(self.device)
            cur.wait_event(ev)
            for v in batch.values():
                if torch.is_tensor(v) and v.is_cuda:
                    v.record_stream(cur)
        self._next = self._stage()  # the next step's copy overlaps this step's compute
        return batch
