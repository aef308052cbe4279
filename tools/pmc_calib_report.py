"""Print every dispatch of a rocprofv3 --pmc run (pmc_calib_random.py) with its
raw counter bytes (FETCH_SIZE / WRITE_SIZE x 1024), in dispatch order.

    python tools/pmc_calib_report.py <pmc_dir> [<pmc_dir> ...]
"""
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_collect import read  # noqa: E402


def main(dirs):
    for d in dirs:
        rows = read(d)
        print(f"== {d}")
        for k in sorted(rows):
            name, cnt, t = rows[k]
            vals = " ".join(f"{c}={v * 1024 / 1e6:.1f}MB" for c, v in sorted(cnt.items()))
            print(f"{k:4d} {t * 1e6:9.1f}us {vals}  {name[:90]}")


if __name__ == "__main__":
    main(sys.argv[1:])
