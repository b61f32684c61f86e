"""The native CSV writer reproduces pandas' output of the decoded frame byte for byte."""
import os

import numpy as np
import pytest

from fed_tgan_amd.data.decode import csv_columns, decode_frame
from fed_tgan_amd.data.vocab import CategoryVocab
from fed_tgan_amd.ops import native
from fed_tgan_amd.utils import csvio


def _table(n=3000, seed=0):
    rng = np.random.default_rng(seed)
    meta = {"columns": [{"column_name": "cat", "type": "categorical"},
                        {"column_name": "bytes", "type": "continous"},
                        {"column_name": "rate", "type": "continous"},
                        {"column_name": "q,uoted", "type": "categorical"}],
            "non_negative_cols": ["bytes"], "date_info": {}}
    vocabs = [CategoryVocab(["tcp", "udp", "empty", "0", "1"]), CategoryVocab(['a,b', 'say "hi"', "plain"])]
    vals = np.stack([rng.integers(0, 5, n), rng.normal(5, 6, n), rng.normal(0, 1, n) * 10.0 ** rng.integers(-6, 18, n),
                     rng.integers(0, 3, n)], 1).astype(np.float64)
    vals[:5, 2] = [0.0, -0.0, 1e16, 1e-5, 123456789.0]
    return meta, vocabs, vals


def test_python_formatter_matches_pandas(tmp_path):
    meta, vocabs, vals = _table(500)
    ref = tmp_path / "ref.csv"
    decode_frame(vals, meta, vocabs).to_csv(ref, index=False)
    names, kinds, vl = csv_columns(meta, vocabs)
    assert csvio.format_table_py(vals, names, kinds, vl) == ref.read_bytes()


@pytest.mark.skipif(not native.available(), reason="native library not built")
def test_native_writer_matches_pandas(tmp_path):
    meta, vocabs, vals = _table(5000)
    ref = tmp_path / "ref.csv"
    out = tmp_path / "out.csv"
    decode_frame(vals, meta, vocabs).to_csv(ref, index=False)
    names, kinds, vl = csv_columns(meta, vocabs)
    csvio.write_table(str(out), vals, names, kinds, vl, threads=4)     # native path (library loaded)
    assert out.read_bytes() == ref.read_bytes()


@pytest.mark.skipif(not native.available(), reason="native library not built")
def test_native_py_float_repr():
    rng = np.random.default_rng(1)
    L = native.lib()
    xs = list(rng.normal(size=200) * 10.0 ** rng.integers(-20, 20, 200)) + [0.1 + 0.2, 1e16, 1e15, 5e-324, -0.0]
    for x in xs:
        assert L.py_float(float(x)) == repr(float(x))


def _date_table(n, seed, date_dic, empty_frac=0.0):
    """(meta, vocabs, decoded values) of a table with date columns, through the real preprocessing path."""
    import pandas as pd
    from fed_tgan_amd.data.table import TablePreprocessor
    from fed_tgan_amd.fed.stats import merge_categorical_metas
    rng = np.random.default_rng(seed)
    base = pd.Timestamp("1993-01-01")
    cols = {"proto": rng.choice(["tcp", "udp", "icmp"], n), "bytes": rng.exponential(500, n).round(),
            "rate": rng.normal(0, 1, n)}
    for c, spec in date_dic.items():
        ts = base + pd.to_timedelta(rng.integers(0, 3 * 365, n), unit="D")
        if "hh" in spec:
            ts = ts + pd.to_timedelta(rng.integers(0, 86400, n), unit="s")
        if spec.startswith("yymmdd|"):
            v = ts.strftime("%y%m%d").astype(int).astype(object)
        else:
            v = ts.strftime("%Y-%m-%d %H:%M:%S" if "hh" in spec else "%Y-%m-%d").astype(object)
        v = pd.Series(v)
        if empty_frac:
            v[rng.random(n) < empty_frac] = np.nan
        cols[c] = v
    df = pd.DataFrame(cols)
    tp = TablePreprocessor(df, "t", "binary_classification", "proto", ["proto"], ["bytes"], date_dic)
    meta, vocabs, _ = merge_categorical_metas([tp.local_meta()])
    enc = tp.encode(vocabs).astype(np.float64)
    # random codes per categorical column (the generator's output space), incl. impossible days
    cursor = 0
    for j, c in enumerate(meta["columns"]):
        if c["type"] == "categorical":
            enc[:, j] = rng.integers(0, len(vocabs[cursor].tolist()), n)
            cursor += 1
    return meta, vocabs, enc


@pytest.mark.skipif(not native.available(), reason="native library not built")
@pytest.mark.parametrize("date_dic,empty", [({"when": "YYYY-MM-DD"}, 0.0), ({"when": "YYYY-MM-DD"}, 0.05),
                                            ({"when": "yymmdd|YYYY-MM-DD"}, 0.0), ({"when": "yymmdd|YYYY-MM-DD"}, 0.05),
                                            ({"at": "YYYY-MM-DD-hh-mm-ss"}, 0.0),
                                            ({"when": "YYYY-MM-DD", "at": "YYYY-MM-DD-hh-mm-ss"}, 0.02),
                                            ({"ym": "YYYY-MM"}, 0.0)])
def test_native_writer_date_columns_match_pandas(tmp_path, date_dic, empty):
    """date schemas keep the native formatter (re-join in csv_writer.cpp), byte for byte."""
    from fed_tgan_amd.data.decode import csv_layout
    meta, vocabs, vals = _date_table(3000, 5, date_dic, empty)
    ref, out = tmp_path / "ref.csv", tmp_path / "out.csv"
    decode_frame(vals, meta, vocabs).to_csv(ref, index=False)
    lay = csv_layout(meta, vocabs)
    assert lay is not None and lay.has_dates
    csvio.write_layout(str(out), vals, lay, threads=4)
    assert out.read_bytes() == ref.read_bytes()


@pytest.mark.skipif(not native.available(), reason="native library not built")
def test_native_writer_midnight_only_times(tmp_path):
    """A time-of-day format whose rows are all midnight prints date-only, as pandas does for datetime64."""
    from fed_tgan_amd.data.decode import csv_layout
    meta, vocabs, vals = _date_table(500, 6, {"at": "YYYY-MM-DD-hh-mm-ss"})
    cursor = 0
    for j, c in enumerate(meta["columns"]):
        if c["type"] == "categorical":
            if c["column_name"].split("-")[-1] in ("hour", "minute", "second"):
                vals[:, j] = vocabs[cursor].tolist().index("00") if "00" in vocabs[cursor].tolist() else vals[0, j]
            cursor += 1
    ref, out = tmp_path / "ref.csv", tmp_path / "out.csv"
    decode_frame(vals, meta, vocabs).to_csv(ref, index=False)
    csvio.write_layout(str(out), vals, csv_layout(meta, vocabs), threads=2)
    assert out.read_bytes() == ref.read_bytes()


@pytest.mark.skipif(not native.available(), reason="native library not built")
def test_native_writer_reports_write_failure(tmp_path):
    """a failed write / close raises instead of leaving a truncated table recorded as written."""
    meta, vocabs, vals = _table(200)
    names, kinds, vl = csv_columns(meta, vocabs)
    with pytest.raises(RuntimeError):
        csvio.write_table(str(tmp_path / "missing_dir" / "x.csv"), vals, names, kinds, vl)
    if os.path.exists("/dev/full"):
        with pytest.raises(RuntimeError, match="short write|close failed"):
            csvio.write_table("/dev/full", np.repeat(vals, 50, axis=0), names, kinds, vl)
