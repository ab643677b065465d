"""Per-kernel duration summary of a rocprofv3 --kernel-trace sqlite output
(run_results.db): count, average and median microseconds per kernel name."""
import collections
import sqlite3
import statistics
import sys


def main(path):
    db = sqlite3.connect(path)
    cur = db.cursor()
    ks = dict(cur.execute("select id, kernel_name from rocpd_info_kernel_symbol"))
    agg = collections.defaultdict(list)
    for kid, s, e in cur.execute("select kernel_id, start, end from rocpd_kernel_dispatch"):
        agg[ks[kid]].append((e - s) / 1000)
    for name, v in sorted(agg.items(), key=lambda x: -sum(x[1])):
        print("%-80s n=%4d avg=%9.2f us med=%9.2f" % (name.split("(")[0][-80:], len(v), sum(v) / len(v),
                                                      statistics.median(v)))


if __name__ == "__main__":
    main(sys.argv[1])
