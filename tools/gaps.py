"""Device idle time between kernels from a rocprofv3 kernel_trace.csv: the union of the
kernels' [start, end) intervals over the traced span, and the largest idle gaps with the
kernels on either side.   python tools/gaps.py <kernel_trace.csv> [--skip-ms 0]"""
import csv
import sys


def main():
    path = sys.argv[1]
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]))
    rows.sort()
    # skip the first half (warmup, first-call allocations)
    rows = rows[len(rows) // 2:]
    t0, busy, cur_s, cur_e, prev = rows[0][0], 0, rows[0][0], rows[0][1], rows[0][2]
    gaps = []
    for s, e, n in rows[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, prev, n))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
        if e >= cur_e:
            prev = n
    busy += cur_e - cur_s
    span = cur_e - t0
    print(f"span {span / 1e3:.1f} us, busy {busy / 1e3:.1f} us, idle {(span - busy) / 1e3:.1f} us "
          f"({100 * (span - busy) / span:.1f} %), {len(gaps)} gaps")
    agg = {}
    for g, a, b in gaps:
        k = (a, b)
        agg.setdefault(k, [0, 0])
        agg[k][0] += g
        agg[k][1] += 1
    for (a, b), (tot, cnt) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:12]:
        print(f"{tot / 1e3:9.1f} us over {cnt:4d} gaps  {a}  ->  {b}")


if __name__ == "__main__":
    main()
