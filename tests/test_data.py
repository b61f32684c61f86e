"""Data layer: meta generation, label encoding, log1p, dates, decode, synthetic generators, sharding."""
import json

import numpy as np
import pandas as pd
import pytest

from fed_tgan_amd.data.date import join_dates, split_dates
from fed_tgan_amd.data.decode import decode_frame
from fed_tgan_amd.data.schema import DatasetSpec, get_spec, intrusion_spec
from fed_tgan_amd.data.synthetic import (generate, generate_adult, generate_covertype, generate_intrusion,
                                         generate_wide, shard)
from fed_tgan_amd.data.table import TablePreprocessor, detect_integer_columns, dump_meta_json
from fed_tgan_amd.data.vocab import CategoryVocab
from fed_tgan_amd.fed.stats import merge_categorical_metas


def _tp(df, spec):
    return TablePreprocessor(df, "Intrusion_train", spec.problem_type, spec.target_column, spec.categorical_list,
                             spec.nonnegative_list, spec.date_dic)


def test_intrusion_generator_schema():
    df = generate_intrusion(3000, seed=1)
    spec = intrusion_spec()
    assert list(df.columns) == spec.selected_variables
    assert (df.dtypes == np.int64).sum() == 23 and (df.dtypes == np.float64).sum() == 15
    assert set(df["protocol_type"]) <= {"tcp", "udp", "icmp"}
    assert df["class"].value_counts().index[0] == "normal."
    assert (df["serror_rate"].between(0, 1)).all()


def test_meta_matches_reference_format():
    spec = intrusion_spec()
    df = generate_intrusion(2000, seed=2)
    meta = _tp(df, spec).local_meta()
    assert set(meta) == {"columns", "problem_type", "name", "date_info", "integer_info", "non_negative_cols", "target"}
    # integer columns exactly as in the reference's Intrusion_train.json
    assert meta["integer_info"] == ["duration", "src_bytes", "dst_bytes", "land", "wrong_fragment", "urgent", "hot",
                                    "num_failed_logins", "logged_in", "num_compromised", "root_shell", "su_attempted",
                                    "num_root", "num_file_creations", "num_shells", "num_access_files",
                                    "num_outbound_cmds", "is_host_login", "is_guest_login", "count", "srv_count",
                                    "dst_host_count", "dst_host_srv_count"]
    col = {c["column_name"]: c for c in meta["columns"]}
    assert col["protocol_type"]["type"] == "categorical"
    assert col["duration"]["type"] == "continous"          # reference spelling
    assert sum(col["service"]["i2s"].values()) == 2000
    assert col["src_bytes"]["max"] == pytest.approx(np.log(df["src_bytes"].max() + 1))
    assert [c["column no"] for c in meta["columns"]] == list(range(42))


def test_encode_with_global_vocab_and_log1p():
    spec = intrusion_spec()
    df = generate_intrusion(1500, seed=3)
    tp = _tp(df, spec)
    meta, vocabs, _ = merge_categorical_metas([tp.local_meta()])
    enc = tp.encode(vocabs)
    j = spec.selected_variables.index("protocol_type")
    assert np.array_equal(vocabs[0].inverse_transform(enc[:, j].astype(int)), df["protocol_type"].astype(str).values)
    k = spec.selected_variables.index("dst_bytes")
    assert np.allclose(enc[:, k], np.log1p(df["dst_bytes"].values))


def test_vocab_matches_sklearn_label_encoder():
    from sklearn.preprocessing import LabelEncoder
    vals = ["b", "a", "10", "2", "a", " ", "Z"]
    v = CategoryVocab(vals)
    le = LabelEncoder().fit(vals)
    assert v.tolist() == le.classes_.tolist()
    assert np.array_equal(v.transform(vals), le.transform(vals))
    assert v.to_sklearn().inverse_transform([0, 2]).tolist() == le.inverse_transform([0, 2]).tolist()
    with pytest.raises(ValueError):
        v.transform(["unseen"])


def test_integer_detection_and_empty():
    df = pd.DataFrame({"a": [1, 2, 3], "b": [1.0, 2.0, np.nan], "c": [1.5, 2.0, 3.0], "d": ["x", " ", "y"]})
    assert detect_integer_columns(df) == ["a", "b"]
    tp = TablePreprocessor(df, "t", "", "", ["d"], [])
    assert tp.df["d"].tolist() == ["x", "empty", "y"]


def test_mixed_object_column_keeps_printed_categories():
    """1, 1.0 and True hash equal but print differently: the categories are what astype(str) gives
    (`Server/dtds/data/utils/file_generator.py:197-205` value_counts of the stringified column)."""
    df = pd.DataFrame({"m": pd.Series([1, 1.0, True, "1", 1, "x"], dtype=object), "v": [1.0, 2, 3, 4, 5, 6]})
    tp = TablePreprocessor(df, "t", "", "", ["m"], [])
    i2s = tp.local_meta()["columns"][0]["i2s"]
    want = df["m"].astype(str).value_counts()
    assert i2s == {str(k): int(v) for k, v in want.items()}
    assert i2s["1"] == 3 and i2s["1.0"] == 1 and i2s["True"] == 1


def test_date_split_join_roundtrip():
    df = pd.DataFrame({"when": ["2020-01-31", "2019-02-15", "empty"], "v": [1, 2, 3]})
    out, cats = split_dates(df, {"when": "YYYY-MM-DD"}, ["when"])
    assert cats == ["when-year", "when-month", "when-day"]
    assert out["when-year"].tolist() == ["20", "19", "empty"]
    back = join_dates(out, {"when": "YYYY-MM-DD"})
    assert back["when"].iloc[2] == "empty"
    assert str(back["when"].iloc[0])[:10] == "2020-01-31"
    # impossible day repaired (Feb 30 -> 28, Apr 31 -> 30)
    bad = pd.DataFrame({"when-year": ["21", "21"], "when-month": ["02", "04"], "when-day": ["30", "31"]})
    fixed = join_dates(bad, {"when": "YYYY-MM-DD"})
    assert [str(x)[5:10] for x in fixed["when"]] == ["02-28", "04-30"]


def test_decode_frame_matches_reference_rules():
    meta = {"columns": [{"column_name": "c", "type": "categorical"}, {"column_name": "n", "type": "continous"},
                        {"column_name": "x", "type": "continous"}],
            "non_negative_cols": ["n"], "date_info": {}}
    vocabs = [CategoryVocab(["a", "empty", "b"])]
    vals = np.array([[0, np.log(3.0), 1.5], [2, -0.5, 2.0], [1, 0.0, 3.0]])
    df = decode_frame(vals, meta, vocabs)
    assert df["c"].tolist() == ["a", " ", "b"]          # codes 0,2,1 of sorted [a, b, empty]
    assert df["n"].iloc[0] == pytest.approx(2.0)
    assert str(df["n"].iloc[1]) == "-0.0"          # ceil of exp(-0.5)-1 keeps the sign like the reference
    assert df["x"].tolist() == [1.5, 2.0, 3.0]


def test_other_generators_and_specs(tmp_path):
    for name, gen in (("adult", generate_adult), ("covertype", generate_covertype)):
        spec = get_spec(name)
        df = gen(500, seed=0)
        assert list(df.columns) == spec.selected_variables
        assert set(spec.categorical_list) <= set(df.columns)
    w = generate_wide(200, n_cols=64)
    assert w.shape == (200, 64)
    spec = intrusion_spec()
    p = tmp_path / "spec.json"
    p.write_text(spec.to_json())
    assert DatasetSpec.from_json(str(p)).categorical_list == spec.categorical_list
    assert generate(get_spec("wide"), 10).shape[1] == 512


@pytest.mark.parametrize("mode", ["iid", "dirichlet", "skew"])
def test_sharding(mode):
    df = generate_intrusion(4000, seed=5)
    parts = shard(df, 4, mode, seed=0, target="class", alpha=0.3)
    assert len(parts) == 4 and all(len(p) > 0 for p in parts)
    if mode != "skew":
        assert sum(len(p) for p in parts) == len(df)
    if mode == "dirichlet":   # label skew: class shares differ across clients
        shares = [p["class"].eq("normal.").mean() for p in parts]
        assert max(shares) - min(shares) > 0.05


def test_meta_json_dump(tmp_path):
    spec = intrusion_spec()
    meta = _tp(generate_intrusion(300, seed=6), spec).local_meta()
    p = tmp_path / "m.json"
    dump_meta_json(meta, str(p))
    again = json.loads(p.read_text())
    assert again["columns"][0]["column_name"] == "duration"


@pytest.mark.parametrize("name", ["intrusion", "adult"])
def test_arrow_reader_matches_pandas(tmp_path, name):
    """read_csv_table(reader="arrow") (pyarrow's parser, dictionary-encoded strings) gives the preprocessor the same
    metadata, vocabulary and encoded matrix as pd.read_csv -- including pandas' missing-value spellings in a
    categorical column."""
    pytest.importorskip("pyarrow")
    from fed_tgan_amd.data.table import read_csv_table
    spec = get_spec(name)
    df = generate(spec, 3000, seed=5)
    cat = spec.categorical_list[0]
    df = df.astype({cat: object})
    df.loc[df.index[5::89], cat] = np.nan               # gaps in a categorical column
    path = tmp_path / "client.csv"
    df.to_csv(path, index=False)
    text = path.read_text().replace(",,", ",NA,", 3)    # pandas' "NA" spelling too
    path.write_text(text)
    tps = [_tp(read_csv_table(str(path), r)[spec.selected_variables], spec) for r in ("pandas", "arrow")]
    m0, m1 = (dict(tp.local_meta()) for tp in tps)
    m0.pop("name"), m1.pop("name")                     # (the reference's per-instance name suffix)
    assert json.dumps(m0, sort_keys=True, default=str) == json.dumps(m1, sort_keys=True, default=str)
    metas = [tps[0].local_meta()]
    _, vocabs, _ = merge_categorical_metas(metas)
    a, b = (tp.encode(vocabs) for tp in tps)
    np.testing.assert_array_equal(np.asarray(a), np.asarray(b))


def test_auto_reader_is_pandas_bitwise(tmp_path):
    """reader="auto" must give pd.read_csv's bits whatever the file size: arrow's correctly rounded
    float parser and pandas' default parser disagree in the last ulp of many random doubles, which would move
    VGM fits and encodings away from the reference's load path (`Server/dtds/data/load.py:51-70`)."""
    pytest.importorskip("pyarrow")
    from fed_tgan_amd.data import table
    rng = np.random.default_rng(0)
    n = 20000
    df = pd.DataFrame({"f": rng.standard_normal(n) * 1e3, "g": np.exp(rng.standard_normal(n) * 5),
                       "i": rng.integers(0, 1000, n).astype(float), "c": rng.choice(["a", "bb", " d"], n)})
    df.loc[rng.random(n) < 0.05, "i"] = np.nan
    path = tmp_path / "t.csv"
    df.to_csv(path, index=False)
    ref = pd.read_csv(path)
    old = table.ARROW_MIN_BYTES
    table.ARROW_MIN_BYTES = 1            # even a "large" file
    try:
        got = table.read_csv_table(str(path), "auto")
    finally:
        table.ARROW_MIN_BYTES = old
    assert list(got.dtypes) == list(ref.dtypes)
    for c in ("f", "g", "i"):
        assert np.array_equal(got[c].to_numpy().view(np.int64), ref[c].to_numpy().view(np.int64)), c
    arrow = table.read_csv_table(str(path), "arrow")
    # (the opt-in arrow reader really does differ in the last bits: why auto must not pick it)
    assert not np.array_equal(arrow["g"].to_numpy(dtype=np.float64), ref["g"].to_numpy())
