"""The native CSV writer reproduces pandas' output of the decoded frame byte for byte."""
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
