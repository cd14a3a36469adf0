"""The step's stream plan: every side stream a training step uses, created once per device in a
fixed order, each on a hardware queue of its own.

HIP multiplexes a process's streams onto ``GPU_MAX_HW_QUEUES`` (4 on the MI355X boxes) pooled
HSA queues; torch's pool streams (``torch.cuda.Stream()``) are handed out round-robin from a pool
of 32 that was spread over those queues when the pool was created.  Which queue a side stream
got therefore depended on how many pool streams had been taken before it, and two streams on one
queue serialise: one extra pool stream taken by the logged-nll overlap moved the reference
schedule's side streams and slowed it from 222 to 240 ms/step (profiles/nll_side_stream_ab_r4.txt).

Here the plan ("ordered", the default) creates its plain streams (``stream_create(mode=0)``,
csrc/runtime/streams.cpp) once per device, before RCCL and torch's pool take any queue
(basic_utils/dist_util.py ``claim_stream_plan`` runs right after ``set_device``): HIP hands a new
stream the least-used queue, so side, wgrad and nll/copy land on queues 2, 3 and 4, and the
compute stream keeps queue 1 (measured from a rocprofv3 trace of the real start-up order,
profiles/stream_queues_r5.txt; bench.py reports it as ``streams.hw_queues_expected``).  A CU-masked
stream (mode 1, plan "cumask") gets a dedicated HSA queue, but the overlapped reference schedule
ran 523-529 ms/step on such streams against ~222 (profiles/stream_plan_ab_r5.txt), so it stays an
A/B option.  Roles (reference call sites whose work they carry; the reference runs everything on
the default stream of its DDP setup, /root/reference/utils/trainer.py:115-128):

=========  ==========================================================================
compute    the current stream (not created here): forward, backward, optimizer
side       second forward/backward stream of the overlapped micro-batch schedule
           (utils/trainer.py ``_forward_backward_overlapped``; reference trainer.py:216-235)
wgrad      deferred weight gradients of the un-armed micro-batches (ops/nn.py deferral)
nll        the logged nll's forward-only vocabulary sweep (models/gaussian_diffusion.py)
copy       H2D prefetch of the next batch (data/prefetch.py; reference trainer.py:210-213)
comm       the data plane: the C++ reducer's bucket all-reduces / reduce-scatters and ZeRO-1
           gathers (csrc/comm/reducer.cpp; reference trainer.py:115-128), on the nll queue
=========  ==========================================================================

Every stream stays on the GPU_MAX_HW_QUEUES pooled queues.  Round 5 gave the reducer a new
highest-priority stream, which HIP puts on a queue of its own; measured on the simulated data
plane (round 6) that fifth queue slowed the overlapped reference schedule from 209 to 229
ms/step while the stand-in comm kernels on a pooled queue cost nothing (CU-masked streams, also
one queue each, had cost far more: 523 ms/step, profiles/stream_plan_ab_r5.txt).

``StreamPlan(device, mode="pool")`` gives torch pool streams, ``"cumask"`` the CU-masked ones (A/B
runs); without the native extension the plan falls back to ``"pool"``."""
import os

import torch

ROLES = ("side", "wgrad", "nll", "copy", "comm")


class StreamPlan:
    _plans = {}

    def __init__(self, device, mode=None):
        self.device = torch.device(device)
        self.mode = mode or "ordered"
        self.streams = {}
        if self.device.type != "cuda":
            return
        ext = None
        if self.mode in ("ordered", "cumask"):
            from ..ops._ext import get_ext
            # required=False: a stock run (use_hip_kernels=False, --stock) needs no native code,
            # and without the extension the plan falls back to torch pool streams
            ext = get_ext(required=False)
            if ext is None or not hasattr(ext, "stream_create"):
                self.mode = "pool"
        with torch.cuda.device(self.device):
            for role in ROLES:  # fixed creation order
                if self.mode == "ordered" and role in ("copy", "comm"):
                    # 4 queues: the brief H2D prefetch and the data plane share the nll queue (an
                    # extra high-priority queue for the data plane cost the overlapped reference
                    # schedule 20 ms/step: profiles/sim_comm_r6.json)
                    s = self.streams["nll"]
                elif self.mode in ("ordered", "cumask"):
                    s = torch.cuda.ExternalStream(ext.stream_create(1 if self.mode == "cumask" else 0, 0),
                                                  device=self.device)
                else:
                    s = torch.cuda.Stream(device=self.device)
                self.streams[role] = s

    @classmethod
    def for_device(cls, device):
        """The process-wide plan of ``device`` (created on first use, never destroyed)."""
        device = torch.device(device)
        if device.type == "cuda" and device.index is None:
            device = torch.device("cuda", torch.cuda.current_device())
        key = (device.type, device.index)
        if key not in cls._plans:
            cls._plans[key] = cls(device)
        return cls._plans[key]

    @staticmethod
    def roles():
        return ROLES

    def get(self, role):
        """The stream of ``role`` (None on CPU)."""
        if role not in ROLES:
            raise KeyError(role)
        return self.streams.get(role)

    # HSA queue of each role EXPECTED for the "ordered" plan: measured once from a rocprofv3 kernel
    # trace of the real start-up order (tools/probes/stream_queues.py, GPU_MAX_HW_QUEUES=4), not
    # re-measured per run (HIP exposes no queue id)
    EXPECTED_QUEUES = {"compute": 1, "side": 2, "wgrad": 3, "nll": 4, "copy": 4, "comm": 4,
                       "zero_gather": "comm",
                       "source": "profiles/stream_queues_r5.txt (one trace, not this run; comm: round 6)"}

    def describe(self):
        d = {"mode": self.mode, "roles": list(ROLES),
             "handles": {r: hex(s.cuda_stream) for r, s in self.streams.items()},
             "gpu_max_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES", "4 (HIP default)")}
        if self.mode == "ordered":
            d["hw_queues_expected"] = dict(self.EXPECTED_QUEUES)
        return d


def plan_stream(device, role):
    """Shorthand: the stream of ``role`` in ``device``'s plan (None on CPU)."""
    if torch.device(device).type != "cuda":
        return None
    return StreamPlan.for_device(device).get(role)
