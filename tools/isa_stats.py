#!/usr/bin/env python3
"""Static instruction mix of every kernel in a gfx950 assembly file.

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=fast -Icsrc/include \
        --cuda-device-only -S -o /tmp/k.s csrc/kernels/fft.hip
    python tools/isa_stats.py /tmp/k.s [name-substring]

Counts straight-line instructions (not dynamic executions): VALU (of which
packed v_pk_*), transcendental, SALU, LDS, global/buffer memory, MFMA, and
the VGPR / SGPR / spill figures from the kernel descriptor metadata.
"""
from __future__ import annotations

import re
import sys

TRANS = ("v_sin_", "v_cos_", "v_exp_", "v_log_", "v_rcp_", "v_rsq_", "v_sqrt_")


def kernels(text: str):
    for m in re.finditer(r"^([A-Za-z_][\w.$]*):\s*; @\1\n(.*?)^\.Lfunc_end", text, re.S | re.M):
        yield m.group(1), m.group(2)


def mix(body: str) -> dict:
    ins = [ln.split()[0] for ln in (l.strip() for l in body.split("\n"))
           if ln and not ln.startswith((".", ";")) and not ln.endswith(":")]
    c = dict(total=len(ins))
    c["valu"] = sum(i.startswith("v_") and not i.startswith("v_mfma") for i in ins)
    c["pk"] = sum(i.startswith("v_pk_") for i in ins)
    c["trans"] = sum(i.startswith(TRANS) for i in ins)
    c["mfma"] = sum(i.startswith("v_mfma") for i in ins)
    c["salu"] = sum(i.startswith("s_") for i in ins)
    c["lds"] = sum(i.startswith("ds_") for i in ins)
    c["vmem"] = sum(i.startswith(("global_", "buffer_", "flat_")) for i in ins)
    c["barrier"] = sum(i == "s_barrier" for i in ins)
    return c


def meta(text: str) -> dict:
    out = {}
    for blk in re.split(r"\n\s+- \.", text.split("amdhsa.kernels:", 1)[-1]):
        name = re.search(r"\.name:\s+(\S+)", blk)
        if not name:
            continue
        g = lambda k: (re.search(rf"\.{k}:\s+(\d+)", blk) or [None, "?"])[1]
        out[name.group(1)] = dict(vgpr=g("vgpr_count"), agpr=g("agpr_count"), sgpr=g("sgpr_count"),
                                  spill=g("vgpr_spill_count"), lds=g("group_segment_fixed_size"))
    return out


def main() -> None:
    text = open(sys.argv[1]).read()
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    md = meta(text)
    for name, body in kernels(text):
        if sub not in name:
            continue
        c = mix(body)
        m = md.get(name, {})
        print(f"{name[:72]}\n  " + " ".join(f"{k}={v}" for k, v in c.items()) + "  " +
              " ".join(f"{k}={v}" for k, v in m.items()))


if __name__ == "__main__":
    main()
