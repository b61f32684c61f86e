"""Epoch-CSV time of a 40,000-row table with date columns: the native formatter (date parts re-joined in
csrc/host/csv_writer.cpp) against the pandas path (decode_frame + to_csv, what date schemas used before).

    python tools/csv_date_probe.py [--rows 40000] [--threads 16]
"""
import argparse
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=40000)
    ap.add_argument("--threads", type=int, default=16)
    args = ap.parse_args()
    from test_csv import _date_table
    from fed_tgan_amd.data.decode import csv_layout, decode_frame
    from fed_tgan_amd.utils import csvio
    d = tempfile.mkdtemp()
    for dic in ({"when": "YYYY-MM-DD"}, {"when": "YYYY-MM-DD", "at": "YYYY-MM-DD-hh-mm-ss"}):
        meta, vocabs, vals = _date_table(args.rows, 0, dic, 0.01)
        lay = csv_layout(meta, vocabs)
        a, b = os.path.join(d, "native.csv"), os.path.join(d, "pandas.csv")
        tn = []
        for _ in range(5):
            t0 = time.perf_counter()
            csvio.write_layout(a, vals, lay, threads=args.threads)
            tn.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        decode_frame(vals, meta, vocabs).to_csv(b, index=False)
        tp = time.perf_counter() - t0
        same = open(a, "rb").read() == open(b, "rb").read()
        print(f"{args.rows} rows, dates {list(dic.values())}: native {min(tn) * 1e3:.1f} ms (best of 5), "
              f"pandas {tp * 1e3:.0f} ms, identical={same}, {os.path.getsize(a) / 1e6:.2f} MB", flush=True)


if __name__ == "__main__":
    main()
