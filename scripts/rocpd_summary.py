"""Summarise a rocprofv3 SQLite (rocpd) output: per-kernel dispatch count and
average duration, or summed PMC counters for kernels matching a pattern.

  python scripts/rocpd_summary.py gpurun_out/<run>/p_results.db [--top 12]
  python scripts/rocpd_summary.py gpurun_out/<run>/p_results.db --pmc --match fbank
"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=12)
    ap.add_argument("--pmc", action="store_true")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    like = f"%{a.match}%"
    if a.pmc:
        q = ("select i.name, sum(p.value), count(distinct d.id) from rocpd_pmc_event p "
             "join rocpd_info_pmc i on p.pmc_id = i.id join rocpd_kernel_dispatch d on d.event_id = p.event_id "
             "join rocpd_info_kernel_symbol s on d.kernel_id = s.id where s.kernel_name like ? group by i.name")
        for name, total, n in c.execute(q, (like,)):
            print(f"{name:28s} {total / max(n, 1):16.1f} per dispatch (n={n})")
        return
    q = ("select s.kernel_name, count(*), avg(d.end - d.start), sum(d.end - d.start) from rocpd_kernel_dispatch d "
         "join rocpd_info_kernel_symbol s on d.kernel_id = s.id where s.kernel_name like ? "
         "group by s.kernel_name order by sum(d.end - d.start) desc limit ?")
    for name, n, avg, tot in c.execute(q, (like, a.top)):
        print(f"{name[:90]:90s} {n:6d} {avg / 1e3:10.1f} us {tot / 1e6:10.3f} ms")


if __name__ == "__main__":
    main()
