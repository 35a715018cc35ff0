"""Summarise rocprofv3 --pmc counter CSVs (scripts/gpu_pmc.sh) per kernel, per dispatch: MFMA
utilisation (busy cycles / SIMD cycles), bf16 MFMA GFLOP (MOPS x 512), LDS bank-conflict rate
(conflict cycles / LDS active cycles), HBM bytes fetched / written, L2 hit rate, and the wave-cycle
split (parked on waitcnt / barrier, issue-stalled, issuing)."""
import csv
import glob
import os
import sys
from collections import defaultdict


def short(name: str) -> str:
    name = name.split("(")[0]
    return name[:60]


def main(root: str) -> None:
    tot = defaultdict(lambda: defaultdict(float))
    nd = defaultdict(set)
    for f in glob.glob(os.path.join(root, "g*", "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = short(r.get("Kernel_Name", "?"))
                tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
                nd[k].add((f, r.get("Dispatch_Id")))
    rows = []
    for k, c in tot.items():
        mf = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        gui = c.get("GRBM_GUI_ACTIVE", 0.0)
        busy = c.get("SQ_BUSY_CU_CYCLES", 0.0)
        lds = c.get("SQ_LDS_IDX_ACTIVE", 0.0)
        bc = c.get("SQ_LDS_BANK_CONFLICT", 0.0)
        rows.append((gui, k, dict(
            # MFMA_BUSY is summed over the 1024 SIMDs; GRBM_GUI_ACTIVE over the 8 XCDs
            mfma_util_pct=100.0 * mf / (1024 * gui / 8) if gui else None,
            mfma_bf16_gflop=c.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0.0) * 512 / 1e9,
            lds_conflict_pct=100.0 * bc / lds if lds else None,
            # FETCH_SIZE / WRITE_SIZE expressions of `rocprofv3 --list-avail` (bytes)
            fetch_MB=(c.get("TCC_BUBBLE_sum", 0.0) * 128
                      + (c.get("TCC_EA0_RDREQ_sum", 0.0) - c.get("TCC_BUBBLE_sum", 0.0)
                         - c.get("TCC_EA0_RDREQ_32B_sum", 0.0)) * 64
                      + c.get("TCC_EA0_RDREQ_32B_sum", 0.0) * 32) / 2 ** 20,
            write_MB=((c.get("TCC_EA0_WRREQ_sum", 0.0) - c.get("TCC_EA0_WRREQ_64B_sum", 0.0)) * 32
                      + c.get("TCC_EA0_WRREQ_64B_sum", 0.0) * 64) / 2 ** 20,
            cu_busy_cycles=busy,
            l2_hit_pct=(100.0 * c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c.get("TCC_MISS_sum", 0.0))
                        if c.get("TCC_HIT_sum") else None),
            # wave-cycle split (disjoint): parked on s_waitcnt / barrier, issue-stalled, issuing
            wait_pct=100.0 * c.get("SQ_WAIT_ANY", 0.0) / c["SQ_WAVE_CYCLES"] if c.get("SQ_WAVE_CYCLES") else None,
            stall_pct=100.0 * c.get("SQ_WAIT_INST_ANY", 0.0) / c["SQ_WAVE_CYCLES"] if c.get("SQ_WAVE_CYCLES") else None,
            active_pct=100.0 * c.get("SQ_ACTIVE_INST_ANY", 0.0) / c["SQ_WAVE_CYCLES"] if c.get("SQ_WAVE_CYCLES") else None)))
    rows.sort(reverse=True)
    # per dispatch: each counter group's run sees every kernel's dispatches once (groups are separate
    # runs of the same program), so the dispatch count of one group divides the sums
    print(f"{'kernel':60s} {'disp':>5s} {'MFMA%':>7s} {'bf16GF/d':>9s} {'LDSconf%':>9s} {'fetchMB/d':>10s} "
          f"{'writeMB/d':>10s} {'L2hit%':>7s} {'wait%':>6s} {'stall%':>7s} {'issue%':>7s}")
    for gui, k, d in rows:
        f = lambda v, fmt: (fmt % v) if v is not None else "-"  # noqa: E731
        n = max(1, len({x for x in nd[k] if "/g1/" in x[0]}) or 1)
        nf = max(1, len({x for x in nd[k] if "/g3/" in x[0]}) or 1)
        nw = max(1, len({x for x in nd[k] if "/g4/" in x[0]}) or 1)
        print(f"{k:60s} {n:5d} {f(d['mfma_util_pct'], '%7.1f')} {d['mfma_bf16_gflop'] / n:9.3f} "
              f"{f(d['lds_conflict_pct'], '%9.2f')} {d['fetch_MB'] / nf:10.2f} {d['write_MB'] / nw:10.2f} "
              f"{f(d['l2_hit_pct'], '%7.1f')} {f(d['wait_pct'], '%6.1f')} {f(d['stall_pct'], '%7.1f')} "
              f"{f(d['active_pct'], '%7.1f')}")


if __name__ == "__main__":
    main(sys.argv[1])
