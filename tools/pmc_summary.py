"""Per-kernel HBM traffic and MFMA utilisation from three rocprofv3 --pmc
passes (FETCH_SIZE; WRITE_SIZE; SQ_INSTS_VALU_MFMA_MOPS_F64|F32 +
SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE), per dispatch.

gfx950: FETCH_SIZE counts 64 B per 128-B request of wide coalesced reads
(MI355X_MICROARCH.md, HBM), so 2x FETCH_SIZE is also printed.  MFMA lines:
MOPS x 512 = counted MFMA flops per dispatch; the utilisation is
SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs): the share of
the dispatch's cycles (GRBM_GUI_ACTIVE is summed over the 8 XCDs) in which
the chip's 256 x 4 matrix pipes were busy.
usage: pmc_summary.py FETCH_DIR WRITE_DIR [MFMA_DIR DTYPE]"""
import csv
import glob
import sys
from collections import defaultdict


def load(d, counter):
    files = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    acc = defaultdict(lambda: [0, 0.0])
    seen = set()
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name", counter) != counter:
                continue
            k = r["Kernel_Name"]
            key = (k, r.get("Dispatch_Id"), r.get("Agent_Id"))
            acc[k][1] += float(r["Counter_Value"])
            if key not in seen:
                seen.add(key)
                acc[k][0] += 1
    return acc


fetch, write = load(sys.argv[1], "FETCH_SIZE"), load(sys.argv[2], "WRITE_SIZE")
print(f"{'kernel':60s} {'disp':>6s} {'FETCH MiB/disp':>15s} {'2xFETCH':>10s} {'WRITE MiB/disp':>15s}")
for k in sorted(fetch, key=lambda k: -fetch[k][1]):
    n, f = fetch[k]
    w = write.get(k, [1, 0.0])
    print(f"{k[:60]:60s} {n:6d} {f / n / 1024:15.3f} {2 * f / n / 1024:10.3f} {w[1] / max(w[0], 1) / 1024:15.3f}")
if len(sys.argv) > 4:
    dt = sys.argv[4]
    mops = load(sys.argv[3], "SQ_INSTS_VALU_MFMA_MOPS_" + ("F64" if dt == "f64" else "F32"))
    busy = load(sys.argv[3], "SQ_VALU_MFMA_BUSY_CYCLES")
    gui = load(sys.argv[3], "GRBM_GUI_ACTIVE")
    print()
    print(f"{'MFMA kernel':60s} {'disp':>6s} {'GFLOP/disp':>11s} {'busy Mcyc':>10s} {'wall kcyc':>10s} {'util':>7s}")
    for k in sorted(mops, key=lambda k: -mops[k][1]):
        n, mo = mops[k]
        if mo <= 0:
            continue
        b = busy.get(k, [1, 0.0])[1] / max(busy.get(k, [1, 0.0])[0], 1)
        g = gui.get(k, [1, 0.0])[1] / max(gui.get(k, [1, 0.0])[0], 1)
        wall = g / 8.0
        util = b / (wall * 1024.0) if wall > 0 else 0.0
        head = k.split("(")[0]
        base = head.split("<")[0].split("::")[-1]                    # e.g. k_rpass
        targs = head[len(head.split("<")[0]):].replace("brd::blk::", "").replace(" ", "")
        short = (base + targs)[:55]                                  # e.g. k_rpass<double,true,FinArgs>
        print(f"MFMA {short:55s} {n:6d} {mo / n * 512 / 1e9:11.3f} {b / 1e6:10.3f} {wall / 1e3:10.1f} {util:7.4f}")
