"""Which HSA queue does each kind of HIP stream land on?  (the stream plan's evidence)

Run under a kernel trace, then summarise the trace (no GPU needed for the second step); the probe
starts a world-1 RCCL process group the way a training job does:

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sq -o sq -- python3 tools/probes/stream_queues.py
    python3 tools/probes/stream_queues.py --trace gpurun_out/sq

The first step launches one small kernel on each stream in a fixed order (synchronising in
between) and writes the order with each stream's hipStreamGetId; the second joins that order
with the trace's (Queue_Id, Stream_Id) per dispatch of the marker kernel.
"""
import csv
import glob
import json
import os
import sys


def probe(out):
    """The real start-up order of a W = 1 RCCL job: dist_util.setup_dist (which claims the
    stream plan before RCCL), a DDPEngine whose C++ reducer owns the direct communicator and
    its comm stream, then other kinds of streams for comparison."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=os.environ.get("SQ_PORT", "29517"), RANK="0",
                      WORLD_SIZE="1", LOCAL_RANK="0")
    import torch

    from basic_utils import dist_util
    from distributed_pipeline_amd.ops._ext import get_ext
    from distributed_pipeline_amd.parallel.ddp import DDPEngine
    from distributed_pipeline_amd.runtime.streams import StreamPlan
    ext = get_ext(required=True)
    x = torch.zeros(1 << 16, device="cuda")
    order = []

    def mark(name, s):
        with torch.cuda.stream(s):
            x.mul_(1.0001)
        torch.cuda.synchronize()
        order.append({"name": name, "handle": hex(s.cuda_stream)})

    mark("default", torch.cuda.current_stream())
    assert dist_util.setup_dist(silent=True)
    plan = StreamPlan.for_device(torch.device("cuda", 0))
    for role in plan.roles():
        mark("plan:" + role, plan.get(role))
    model = torch.nn.Linear(256, 256).cuda()
    eng = DDPEngine(model, bucket_cap_mb=1.0, first_bucket_mb=0.25)
    comm = eng._native.comm_stream() if eng._native is not None else 0
    if comm:
        mark("reducer_comm", torch.cuda.ExternalStream(comm))
    for i in range(4):
        mark(f"pool{i}", torch.cuda.Stream())
    mark("plain", torch.cuda.ExternalStream(ext.stream_create(0, 0)))
    least, greatest = torch.cuda.Stream.priority_range()
    mark("prio_greatest", torch.cuda.ExternalStream(ext.stream_create(2, greatest)))
    mark("default_again", torch.cuda.current_stream())
    with open(out, "w") as f:
        json.dump({"order": order, "plan": plan.describe(), "direct_reducer": bool(comm)}, f, indent=1)
    print(json.dumps(order))
    del eng
    import torch.distributed as dist
    dist.destroy_process_group()


def summarise(d):
    with open(os.path.join(d, "order.json")) as f:
        info = json.load(f)
    order = info["order"]
    rows = []
    for p in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            if "MulFunctor" in r.get("Kernel_Name", "") or "mul" in r.get("Kernel_Name", "").lower():
                rows.append(r)
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    print(f"# stream -> HSA queue ({len(rows)} marker dispatches, {len(order)} streams)")
    queues = {}
    for o, r in zip(order, rows):
        q = r.get("Queue_Id", "?")
        queues.setdefault(q, []).append(o["name"])
        print(f"{o['name']:16s} handle {o['handle']:>16}  trace Stream_Id {r.get('Stream_Id', '?'):>4}  Queue_Id {q}")
    print("# queues:")
    for q, names in queues.items():
        print(f"  queue {q}: {', '.join(names)}")
    print("# plan:", json.dumps(info["plan"]))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--trace":
        summarise(sys.argv[2])
    else:
        out = os.environ.get("SQ_OUT", "gpurun_out/sq/order.json")
        os.makedirs(os.path.dirname(out), exist_ok=True)
        probe(out)
