"""Static instruction mix of device kernels from a hipcc -S listing.
  hipcc ... --cuda-device-only -S -o /tmp/yk.s core_amd/csrc/yk_device.hip
  python tools/isa_mix.py /tmp/yk.s k_shade_bounce [--blocks]
Counts per class (f64 VALU, other VALU, SALU, VMEM, LDS, branch) for every
kernel whose mangled name contains the pattern; --blocks prints the same per
basic block (label), to find the heavy loops."""
import collections
import re
import sys


def classify(op):
    if op.startswith("v_"):
        return "v_f64" if "f64" in op else "valu"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    return "other"


def main():
    path, pat = sys.argv[1], sys.argv[2]
    blocks = "--blocks" in sys.argv
    lines = open(path).read().split("\n")
    i = 0
    while i < len(lines):
        m = re.match(r"^(_Z\S*" + re.escape(pat) + r"\S*):", lines[i])
        if not m:
            i += 1
            continue
        name = m.group(1)
        tot = collections.Counter()
        per = collections.OrderedDict()
        cur = "entry"
        per[cur] = collections.Counter()
        i += 1
        while i < len(lines) and not lines[i].startswith(".Lfunc_end"):
            l = lines[i]
            lm = re.match(r"^(\.LBB\S+):", l)
            if lm:
                cur = lm.group(1)
                per[cur] = collections.Counter()
            elif l.startswith("\t") and not l.strip().startswith((".", ";")) and l.strip():
                c = classify(l.split()[0])
                tot[c] += 1
                per[cur][c] += 1
            i += 1
        print(f"{name[:70]}  total {sum(tot.values())}  {dict(tot)}")
        if blocks:
            for b, c in per.items():
                if sum(c.values()):
                    print(f"   {b:16s} {sum(c.values()):5d}  {dict(c)}")


if __name__ == "__main__":
    main()
