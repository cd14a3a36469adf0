"""Which HSA queue does each kind of HIP stream land on?  (the stream plan's evidence)

Run under a kernel trace, then summarise the trace (no GPU needed for the second step):

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
    import torch

    from distributed_pipeline_amd.ops._ext import get_ext
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
    plan = StreamPlan(torch.device("cuda", 0))   # the trainer's plan: created before any pool stream
    for role in plan.roles():
        mark("plan:" + role, plan.get(role))
    for i in range(6):
        mark(f"pool{i}", torch.cuda.Stream())
    for i in range(2):
        mark(f"pool_high{i}", torch.cuda.Stream(priority=-1))
    for i in range(2):
        mark(f"plain{i}", torch.cuda.ExternalStream(ext.stream_create(0, 0)))
    for i in range(2):
        mark(f"cumask{i}", torch.cuda.ExternalStream(ext.stream_create(1, 0)))
    least, greatest = torch.cuda.Stream.priority_range()
    mark("prio_greatest", torch.cuda.ExternalStream(ext.stream_create(2, greatest)))  # the reducer's kind
    mark("default_again", torch.cuda.current_stream())
    with open(out, "w") as f:
        json.dump({"order": order, "plan": plan.describe()}, f, indent=1)
    print(json.dumps(order))


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
        sys.stdout.flush()
        os._exit(0)  # skip static teardown: under rocprofv3 the process segfaulted in exit handlers
