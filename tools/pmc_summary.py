"""Per-launch HBM traffic of a kernel from two rocprofv3 --pmc passes
(FETCH_SIZE, WRITE_SIZE; KB units), with the gfx950 correction of
/opt/skills/guides/MI355X_MICROARCH.md (HBM section): FETCH_SIZE counts half the
bytes of wide coalesced reads, so it is doubled; WRITE_SIZE is exact for 16-B
lanes. Writes a JSON summary that bench.py reports as roofline.traffic.

    python tools/pmc_summary.py FETCH.csv WRITE.csv k_obs out.json [config]
"""
import csv
import json
import statistics
import sys


def per_dispatch(path, name_part, counter):
    vals = []
    for r in csv.DictReader(open(path)):
        if name_part in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals.append(float(r["Counter_Value"]) * 1024.0)
    return vals


def main():
    fetch_csv, write_csv, kernel, out = sys.argv[1:5]
    config = sys.argv[5] if len(sys.argv) > 5 else "c2"
    f = per_dispatch(fetch_csv, kernel, "FETCH_SIZE")
    w = per_dispatch(write_csv, kernel, "WRITE_SIZE")
    fm, wm = statistics.median(f), statistics.median(w)
    summary = {
        "kernel": kernel, "config": config, "dispatches": [len(f), len(w)],
        "fetch_bytes_raw": fm, "fetch_bytes_corrected": 2.0 * fm, "write_bytes": wm,
        "traffic_bytes_per_launch": 2.0 * fm + wm,
        "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes (KB -> bytes), "
                  "FETCH_SIZE x2 (gfx950 correction), median over dispatches",
    }
    json.dump(summary, open(out, "w"), indent=1)
    print(json.dumps(summary))


if __name__ == "__main__":
    main()
