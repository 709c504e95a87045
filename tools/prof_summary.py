#!/usr/bin/env python3
"""Summarise rocprofv3 SQLite output (kernel trace + PMC) into a text table.

    python tools/prof_summary.py gpurun_out/prof/run_results.db [more.db ...] > profiles/x.txt
"""
import sqlite3
import sys
from collections import defaultdict


def summarize(path):
    c = sqlite3.connect(path)
    out = [f"# {path}"]
    q = """select s.kernel_name, count(*), avg(d.end-d.start)/1000.0, min(d.end-d.start)/1000.0,
                  max(d.end-d.start)/1000.0, s.arch_vgpr_count, s.sgpr_count, s.group_segment_size,
                  s.private_segment_size, d.grid_size_x, d.grid_size_y, d.workgroup_size_x
           from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id=s.id
           group by s.kernel_name order by 3*count(*) desc"""
    out.append(f"{'kernel':70s} {'n':>4s} {'avg_us':>9s} {'min_us':>9s} {'max_us':>9s} vgpr sgpr lds scratch grid")
    for r in c.execute(q):
        out.append(f"{r[0][:70]:70s} {r[1]:4d} {r[2]:9.1f} {r[3]:9.1f} {r[4]:9.1f} {r[5]:4} {r[6]:4} {r[7]:5} {r[8]:3} "
                   f"{r[9]}x{r[10]}/{r[11]}")
    try:
        # one row per (dispatch, counter, hardware instance): sum the instances of a
        # dispatch, then average over the dispatches of a kernel
        q2 = """select s.kernel_name, i.name, d.id, sum(p.value)
                from rocpd_pmc_event p join rocpd_info_pmc i on p.pmc_id=i.id
                join rocpd_kernel_dispatch d on d.event_id=p.event_id
                join rocpd_info_kernel_symbol s on d.kernel_id=s.id
                group by s.kernel_name, i.name, d.id"""
        rows = list(c.execute(q2))
        if rows:
            out.append("\n# PMC (sum over hardware instances, average over dispatches)")
            acc = defaultdict(lambda: defaultdict(list))
            for k, n, _, v in rows:
                acc[k][n].append(v)
            for k, per in acc.items():
                out.append(k[:90])
                for n in sorted(per):
                    vals = per[n]
                    out.append(f"    {n:28s} {sum(vals) / len(vals):18.1f}   (n={len(vals)})")
    except sqlite3.Error as e:
        out.append(f"(no pmc: {e})")
    return "\n".join(out)


if __name__ == "__main__":
    for p in sys.argv[1:]:
        print(summarize(p))
        print()
