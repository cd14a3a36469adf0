"""Instruction mix of one kernel in a gfx950 assembly listing (hipcc --cuda-device-only -S):

    python tools/asm_mix.py FILE.s MANGLED_NAME_SUBSTRING [top]
"""
import collections
import sys


def main():
    path, pat = sys.argv[1], sys.argv[2]
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    s = open(path).read()
    names = [l.split(":")[0] for l in s.split("\n")
             if pat in l and not l.startswith((".", "\t", " ", ";")) and ":" in l and "@" in l]
    for name in names:
        i = s.index(name + ":")
        j = s.index(".Lfunc_end", i)
        ins = [l.split()[0] for l in s[i:j].split("\n")[1:]
               if l.strip() and not l.strip().startswith((".", ";", "//")) and not l.strip().endswith(":")]
        c = collections.Counter(ins)
        valu = sum(v for k, v in c.items() if k.startswith("v_") and not k.startswith("v_mfma"))
        print(f"{name}: {len(ins)} instructions, {valu} VALU, {c.get('v_mfma_f32_16x16x32_bf16', 0)} MFMA")
        print("  " + ", ".join(f"{k} {v}" for k, v in c.most_common(top)))


if __name__ == "__main__":
    main()
