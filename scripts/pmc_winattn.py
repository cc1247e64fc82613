"""HBM traffic of the window-attention forward kernel from rocprofv3 PMC counters.

    rocprofv3 --pmc FETCH_SIZE --kernel-trace -d <dirF> -o run -- python3 scripts/pmc_winattn.py run
    rocprofv3 --pmc WRITE_SIZE --kernel-trace -d <dirW> -o run -- python3 scripts/pmc_winattn.py run
    python3 scripts/pmc_winattn.py parse <dirF> <dirW> > profiles/pmc_winattn_fwd.json

`run` issues exactly the 24 irads_winattn_fwd launches of one bench step (Swin-B at 512²,
rgb+dte batched: B = 16; depths 2/2/18/2, shift 0/6 alternating), on the same synthetic
scale as bench.py, after one untimed pass of the same sequence.  Every launch reads its OWN qkv
tensor, as the step's blocks do (round 3's runner reused one per stage, so the 18 stage-2
launches found their inputs in the 256 MB Infinity Cache: FETCH read low).  `parse` takes the last 24
dispatches of the kernel and applies MI355X_MICROARCH.md's gfx950 corrections: FETCH_SIZE
counts half the bytes of wide (16 B/lane) streaming reads, so it is doubled; WRITE_SIZE is
exact for 16 B/lane stores.  Both counters are in KiB.  FETCH_SIZE and WRITE_SIZE need
separate passes (TCC slots: 3 + 2 > 4).
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KIND = os.environ.get("IRADS_PMC_KIND", "fwd")  # fwd | bwd: which window-attention kernel is counted
STAGES = ((128, 128, 4, 2), (64, 256, 8, 2), (32, 512, 16, 18), (16, 1024, 32, 2))  # side, C, heads, depth


def run():
    sys.path.insert(0, os.path.join(ROOT, "ir-ads_amd"))
    import torch
    from irads import ops
    B = 16
    ins = []
    for side, C, nH, depth in STAGES:
        L = side * side
        qkvs = [(torch.randn(B, L, 3 * C, device="cuda") * 0.5).bfloat16() for _ in range(depth)]
        bias = torch.randn(3 * C, device="cuda") * 0.1
        table = torch.randn(23 * 23, nH, device="cuda") * 0.1
        ins.append((qkvs, bias, table, side, nH, depth))

    def step():
        for qkvs, bias, table, side, nH, depth in ins:
            for blk in range(depth):
                ops.winattn_fwd(qkvs[blk], bias, table, None, side, side, nH, 6 if blk % 2 else 0, 32 ** -0.5)

    def step_bwd():  # the 24 backward launches, each on its own forward's output and LSE
        for qkvs, bias, table, side, nH, depth in ins:
            for blk in range(depth):
                shift = 6 if blk % 2 else 0
                qq = qkvs[blk].clone().requires_grad_()
                o = ops.window_attention(qq, bias, table, None, side, side, nH, shift, 32 ** -0.5)
                o.backward(torch.ones_like(o))
    if KIND == "bwd":
        step_bwd()
        step_bwd()
    else:
        step()
        step()
    torch.cuda.synchronize()


def algorithmic_bytes():
    tot = 0
    for side, C, nH, depth in STAGES:
        Np = (-(-side // 12) * 12) ** 2
        # read q, k, v + write o per padded token (fwd); read q, k, v, o, dO + write dq, dk, dv (bwd)
        tot += depth * 16 * Np * (4 if KIND == "fwd" else 8) * C * 2
    return tot / 24


def _values(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    vals = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if f"winattn_{KIND}" in r.get("Kernel_Name", "") and r.get("Counter_Name") == counter:
                    vals.append((int(r.get("Dispatch_Id", 0)), float(r["Counter_Value"])))
    vals.sort()
    return [v for _, v in vals][-24:]


def parse(dir_fetch, dir_write):
    fetch = _values(dir_fetch, "FETCH_SIZE")
    write = _values(dir_write, "WRITE_SIZE")
    if len(fetch) != 24 or len(write) != 24:
        raise SystemExit(f"expected 24 dispatches per counter, got {len(fetch)} / {len(write)}")
    kib = 1024.0
    read_b = 2.0 * sum(fetch) / 24 * kib  # gfx950: FETCH_SIZE = half the bytes of 16-B/lane reads
    write_b = sum(write) / 24 * kib
    out = {"kernel": f"irads_winattn_{KIND} (bf16)", "launches": 24,
           "fetch_size_kib_per_launch_raw": sum(fetch) / 24, "write_size_kib_per_launch": sum(write) / 24,
           "hbm_read_bytes_per_launch": round(read_b), "hbm_write_bytes_per_launch": round(write_b),
           "hbm_bytes_per_launch": round(read_b + write_b),
           "algorithmic_bytes_per_launch": round(algorithmic_bytes()),
           "correction": "FETCH_SIZE x2 (gfx950 counts half of 16-B/lane streaming reads), WRITE_SIZE as is; "
                         "MI355X_MICROARCH.md §HBM",
           "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE --kernel-trace, separate passes, "
                     "scripts/pmc_winattn.py run (the 24 launches of one bench step)"}
    out["traffic_over_algorithmic"] = round(out["hbm_bytes_per_launch"] / out["algorithmic_bytes_per_launch"], 3)
    print(json.dumps(out, indent=1))


SQ_COUNTERS = ("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
               "SQ_ACTIVE_INST_LDS", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CYCLES")


def parse_sq(dir_sq, *counters):
    """Wave-state breakdown of the 24 launches (one SQ pass, 8 counters): SQ_WAIT_ANY =
    parked at s_waitcnt / barrier, SQ_WAIT_INST_ANY = issue-stalled, SQ_ACTIVE_INST_ANY =
    issuing; the three are disjoint and sum to SQ_WAVE_CYCLES (MI355X_MICROARCH.md, PMC
    slots).  The wave counters are in quad-cycles, SQ_VALU_MFMA_BUSY_CYCLES in cycles."""
    names = counters or SQ_COUNTERS
    vals = {c: _values(dir_sq, c) for c in names}
    tot = {c: sum(v) for c, v in vals.items()}
    out = {"kernel": f"irads_winattn_{KIND} (bf16)", "launches": 24,
           "per_launch": {c: round(v / 24) for c, v in tot.items()},
           # dispatch order: stage 0 x2, stage 1 x2, stage 2 x18, stage 3 x2 (shift 0 / 6 alternating)
           "per_stage_sum": {c: [round(sum(v[a:b])) for a, b in ((0, 2), (2, 4), (4, 22), (22, 24))]
                             for c, v in vals.items()},
           "source": "rocprofv3 --pmc " + " ".join(names) + " --kernel-trace, "
                     "scripts/pmc_winattn.py run (the 24 launches of one bench step)"}
    if "SQ_WAVE_CYCLES" in tot:
        w = tot["SQ_WAVE_CYCLES"]
        out["fraction_of_wave_cycles"] = {c: round(tot[c] / w, 3) for c in SQ_COUNTERS[1:6] if c in tot}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    elif sys.argv[1] == "parse_sq":
        parse_sq(sys.argv[2], *sys.argv[3:])
    else:
        parse(sys.argv[2], sys.argv[3])
