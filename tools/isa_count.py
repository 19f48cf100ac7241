#!/usr/bin/env python
"""Static instruction counts of one kernel's innermost loop in a device assembly listing.

    hipcc --offload-arch=gfx950 -O3 ... --cuda-device-only -S gsr_forward.hip -o fwd.s
    python tools/isa_count.py fwd.s render_fwd_v5_kernelILi2ELi8ELb1E

Finds the kernel's label, takes every basic block that belongs to a loop of the deepest nesting depth (the
"in Loop: Header=... Depth=N" annotations), and prints VALU / transcendental / packed / SALU / LDS counts plus a
weighted VALU issue cost (plain 1, v_pk_* 1.7, transcendental 2.7: tools/probes/valu_rate_probe.hip on MI355X).
"""
import re
import sys

TRANS = ("v_exp_f32", "v_rcp_f32", "v_log_f32", "v_sqrt_f32", "v_rsq_f32", "v_sin_f32", "v_cos_f32",
         "v_rcp_iflag_f32")


def main():
    path, sym = sys.argv[1], sys.argv[2]
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\w*" + re.escape(sym) + r"\w*:", l))
    end = next((i for i in range(start + 1, len(lines)) if lines[i].startswith("\t.section") or
                re.match(r"^\.Lfunc_end", lines[i])), len(lines))
    body = lines[start:end]
    # basic blocks with their loop depth
    blocks, cur, depth = [], [], 0
    for l in body:
        m = re.match(r"^(\.LBB\w+|; %bb\.\d+):", l)
        if m:
            blocks.append((depth, cur))
            cur = []
            d = re.search(r"Depth=(\d+)", l)
            depth = int(d.group(1)) if d else 0
            continue
        if l.strip().startswith(";") and "Depth=" in l:
            d = re.search(r"Depth=(\d+)", l)
            depth = int(d.group(1))
            continue
        cur.append(l.strip())
    blocks.append((depth, cur))
    dmax = max(d for d, _ in blocks)
    ins = [l for d, b in blocks if d == dmax for l in b if l and not l.startswith(";") and not l.startswith(".")]
    valu = [l for l in ins if l.startswith("v_")]
    trans = [l for l in valu if l.split()[0].rsplit("_e", 1)[0] in TRANS or l.split()[0] in TRANS]
    pk = [l for l in valu if l.startswith("v_pk_")]
    salu = [l for l in ins if l.startswith("s_") and not l.startswith("s_waitcnt") and not l.startswith("s_nop")]
    lds = [l for l in ins if l.startswith("ds_")]
    cost = len(valu) + 0.7 * len(pk) + 1.7 * len(trans)
    print(f"{sym}: loop depth {dmax}: VALU {len(valu)} (trans {len(trans)}, packed {len(pk)}), weighted {cost:.1f}; "
          f"SALU {len(salu)}; LDS {len(lds)}")
    ops = {}
    for l in valu:
        op = l.split()[0]
        ops[op] = ops.get(op, 0) + 1
    print("  " + ", ".join(f"{k} {v}" for k, v in sorted(ops.items(), key=lambda kv: -kv[1])))


if __name__ == "__main__":
    main()
