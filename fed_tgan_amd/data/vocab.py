"""Label vocabularies (sklearn ``LabelEncoder`` semantics without the sklearn object).

The reference fits one sklearn ``LabelEncoder`` per categorical column on the
frequency-sorted global vocabulary (`Server/dtds/distributed.py:621-624`): codes are the
positions in the *lexicographically* sorted unique string list.  ``CategoryVocab`` keeps
exactly that mapping as a plain sorted ``numpy`` string array so it can be broadcast
as a list over the control plane and used inside native decode kernels; it converts
to / from sklearn ``LabelEncoder`` objects for the ``label_encoders_{name}.pickle`` artefact.
"""
from __future__ import annotations

from typing import Iterable, List, Sequence

import numpy as np


class CategoryVocab:
    __slots__ = ("column_name", "classes_")

    def __init__(self, classes: Iterable[str], column_name: str = ""):
        arr = np.asarray([str(c) for c in classes], dtype=object)
        self.classes_ = np.asarray(sorted(set(arr.tolist())), dtype=object)
        self.column_name = column_name

    # --- LabelEncoder-compatible surface -------------------------------------------------
    def transform(self, values: Sequence) -> np.ndarray:
        import pandas as pd
        vals = pd.Series(values, dtype=object) if not isinstance(values, pd.Series) else values
        if vals.dtype != object or not all(isinstance(v, str) for v in vals.iloc[:64]):
            vals = vals.astype(str)
        idx = pd.Index(self.classes_).get_indexer(vals.to_numpy(dtype=object))   # hash lookup
        if np.any(idx < 0):
            bad = vals.to_numpy(dtype=object)[idx < 0]
            raise ValueError(f"y contains previously unseen labels: {sorted(set(bad.tolist()))[:5]}")
        return idx.astype(np.int64)

    def inverse_transform(self, codes: Sequence) -> np.ndarray:
        codes = np.asarray(codes, dtype=np.int64)
        return self.classes_[codes]

    def __len__(self) -> int:
        return len(self.classes_)

    def tolist(self) -> List[str]:
        return self.classes_.tolist()

    def to_sklearn(self):
        from sklearn.preprocessing import LabelEncoder
        le = LabelEncoder()
        le.classes_ = np.asarray(self.classes_.tolist())
        return le

    @classmethod
    def from_sklearn(cls, le, column_name: str = "") -> "CategoryVocab":
        return cls(le.classes_.tolist(), column_name)

    def __repr__(self) -> str:
        return f"CategoryVocab({self.column_name!r}, n={len(self)})"


def write_label_encoders(path: str, vocabs: Sequence[CategoryVocab]) -> str:
    """``label_encoders_{name}.pickle``: a list of ``{column_name, label_encoder}`` with sklearn
    ``LabelEncoder`` objects (`Server/dtds/distributed.py:669-684`).  Written to a temporary name and
    renamed, so a reader never sees a partial file."""
    import os
    import pickle
    les = [{"column_name": v.column_name, "label_encoder": v.to_sklearn()} for v in vocabs]
    tmp = f"{path}.tmp{os.getpid()}"
    with open(tmp, "wb") as f:
        pickle.dump(les, f, protocol=pickle.HIGHEST_PROTOCOL)
    os.replace(tmp, path)
    return path


if __name__ == "__main__":
    # helper process of the federated runtime (fed/runtime.py start_label_encoders): the sklearn import
    # and the pickle happen here, off the federator's critical path.  stdin: {"path", "vocabs": [[name, classes]]}
    import json
    import os
    import sys
    os.nice(19)          # the federator's rounds run meanwhile: this process only takes idle CPU time
    req = json.load(sys.stdin)
    write_label_encoders(req["path"], [CategoryVocab(c, n) for n, c in req["vocabs"]])
