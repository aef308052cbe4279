"""FETCH_SIZE / WRITE_SIZE calibration for scattered small accesses.

    rocprofv3 --pmc FETCH_SIZE -d <dir> -- python3 tools/pmc_calib_random.py
    rocprofv3 --pmc WRITE_SIZE -d <dir> -- python3 tools/pmc_calib_random.py

MI355X_MICROARCH.md §HBM: FETCH_SIZE reads 1/2 of the bytes of a wide
coalesced stream on gfx950, and "other access widths are uncalibrated:
calibrate on a known byte count in your own access pattern".  The lookup
kernels read 64-128 B pieces of random rows, so this probe runs, in order:
  1. a 1 GiB clone (the streaming calibration tools/pmc_collect.py uses);
  2. index_select of N random DISTINCT rows of R bytes from a 4 GiB table
     (larger than the 256 MiB Infinity Cache, every row read once) for
     R = 64, 128, 256 B, rows R-aligned -- known bytes N*R each;
  3. index_copy_ of the same rows back into the table (scattered writes).
tools/pmc_calib_report.py divides each dispatch's counter by its known bytes.
"""
import torch


def main():
    dev = torch.device("cuda", 0)
    big = torch.empty(1 << 28, device=dev).fill_(1.0)
    big.clone()                                           # 1: 1 GiB streaming read + write
    del big
    table_bytes = 4 << 30
    for R in (64, 128, 256):
        cols = R // 4
        table = torch.ones(table_bytes // R, cols, device=dev)
        n = 1 << 22                                       # 4 Mi rows
        g = torch.Generator(device=dev).manual_seed(R)
        idx = torch.randperm(table.shape[0], device=dev, generator=g)[:n]
        torch.cuda.synchronize()
        rows = table.index_select(0, idx)                 # 2: n*R bytes of scattered reads
        table.index_copy_(0, idx, rows)                   # 3: n*R bytes of scattered writes
        torch.cuda.synchronize()
        print(f"R={R}: rows={n} known_bytes={n * R}")
        del table, rows, idx
    print("probe done")


if __name__ == "__main__":
    main()
