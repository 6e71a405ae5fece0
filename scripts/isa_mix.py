#!/usr/bin/env python3
"""Static instruction mix of one kernel in a device assembly listing
(diagnostic): per basic block, the VALU / SALU / LDS / VMEM / branch counts and
the backward branches (loops), so a VALU-bound kernel's instruction budget can
be split by phase.

    hipcc --offload-arch=gfx950 -O3 ... --offload-device-only -S -o sa.s sparc_amp.hip
    python scripts/isa_mix.py sa.s '_ZN12_GLOBAL__N_16k_secbIfLi8ELi4ELi16ELb1EEEvNS_7SecArgsIT_EE'
"""
import collections
import re
import sys


def kind(op):
    if op.startswith(("v_mfma", "v_smfmac")):
        return "mfma"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith(("s_load", "s_buffer_load")):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    path, fn = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(fn + ":"))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
    blocks, cur = [], ["entry", collections.Counter(), [], start]
    for i in range(start + 1, end):
        l = lines[i].split(";")[0].strip()
        if not l:
            continue
        m = re.match(r"^(\.LBB\S+):$", l)
        if m:
            blocks.append(cur)
            cur = [m.group(1), collections.Counter(), [], i]
            continue
        if l.startswith("."):
            continue
        op = l.split()[0]
        k = kind(op)
        cur[1][k] += 1
        if k == "valu":
            cur[1]["v:" + op] += 1
        if k == "branch":
            tgt = l.split()[-1]
            cur[2].append(tgt)
    blocks.append(cur)
    order = {b[0]: j for j, b in enumerate(blocks)}
    tot = collections.Counter()
    for j, (name, c, br, ln) in enumerate(blocks):
        tot.update({k: v for k, v in c.items() if ":" not in k})
        back = [t for t in br if t in order and order[t] <= j]
        tag = f"  <- loop back to {','.join(back)}" if back else ""
        print(f"{name:16s} line {ln:7d}  valu {c['valu']:4d} lds {c['lds']:3d} vmem {c['vmem']:3d} "
              f"salu {c['salu']:3d} wait {c['wait']:3d}{tag}")
    print("total", dict(tot))
    if len(sys.argv) > 3:  # VALU opcode histogram of the named blocks
        c = collections.Counter()
        for name, cc, _, _ in blocks:
            if name in sys.argv[3:]:
                c.update({k[2:]: v for k, v in cc.items() if k.startswith("v:")})
        for op, v in c.most_common(40):
            print(f"  {op:28s} {v}")


if __name__ == "__main__":
    main()
