"""Static check of a gfx950 asm listing (hipcc -S): an instruction that reads a VGPR written by
an inline-asm LDS read (ds_read_*) before an s_waitcnt lgkmcnt retires that read is a hazard
(the hardware does not interlock LDS returns).  Kernels that issue their fragment reads from asm
(csrc/gemm256.hip, csrc/wgrad4w.hip) rely on the compiler placing the outputs straight into the
MFMA operand registers; this flags any copy or spill of a register still in flight.

    python tools/probes/lds_read_hazards.py kernel.s [function-substring]
"""
import re
import sys


def regs(tok):
    m = re.match(r"([va])\[(\d+):(\d+)\]", tok)
    if m:
        return {f"{m.group(1)}{i}" for i in range(int(m.group(2)), int(m.group(3)) + 1)}
    m = re.match(r"([va])(\d+)$", tok)
    return {tok} if m else set()


def check(path, fn=None):
    bad, pending = [], []  # pending: list of sets of registers, oldest first
    active = fn is None
    for ln, line in enumerate(open(path), 1):
        s = line.split(";")[0].strip()
        if s.endswith(":") and not s.startswith("."):
            active = fn is None or fn in s
            pending = []
            continue
        if not active or not s or s.startswith("."):
            continue
        op = s.split()[0]
        ops = [t.strip() for t in s[len(op):].split(",")]
        if op == "s_waitcnt":
            m = re.search(r"lgkmcnt\((\d+)\)", s)
            if m:
                k = int(m.group(1))
                pending = pending[len(pending) - k:] if k else []
            continue
        dst = regs(ops[0]) if ops and ops[0] else set()
        srcs = set()
        for t in ops[1:] if op.startswith(("v_", "ds_", "scratch_", "buffer_", "global_")) else ops:
            srcs |= regs(t.split()[0]) if t else set()
        if op.startswith(("scratch_store", "global_store", "buffer_store")):
            srcs |= regs(ops[1]) if len(ops) > 1 else set()
        live = set().union(*pending) if pending else set()
        hit = srcs & live
        if hit:
            bad.append((ln, s, sorted(hit)[:4]))
        if op.startswith("ds_read"):
            pending.append(dst)
        elif dst:
            pending = [p - dst for p in pending]
    return bad


if __name__ == "__main__":
    res = check(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
    for ln, s, h in res[:20]:
        print(f"{ln}: {s}   <- in flight: {h}")
    print(f"{len(res)} hazard(s)")
    sys.exit(1 if res else 0)
