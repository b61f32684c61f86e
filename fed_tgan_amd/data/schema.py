"""Dataset specifications (what the reference hard-codes as argparse list defaults).

The reference bakes the Intrusion (KDD-99) schema into `type=list` argparse defaults of
`Server/dtds/distributed.py:916-934` (which cannot really be overridden from a shell).
Here a `DatasetSpec` carries the same information and can be loaded from a JSON file
(`-config spec.json`), so Adult / Covertype / wide tables work through the same CLI.
"""
from __future__ import annotations

import dataclasses
import json
from typing import Dict, List, Optional


INTRUSION_COLUMNS = [
    "duration", "protocol_type", "service", "flag", "src_bytes", "dst_bytes", "land",
    "wrong_fragment", "urgent", "hot", "num_failed_logins", "logged_in", "num_compromised",
    "root_shell", "su_attempted", "num_root", "num_file_creations", "num_shells",
    "num_access_files", "num_outbound_cmds", "is_host_login", "is_guest_login", "count",
    "srv_count", "serror_rate", "srv_serror_rate", "rerror_rate", "srv_rerror_rate",
    "same_srv_rate", "diff_srv_rate", "srv_diff_host_rate", "dst_host_count",
    "dst_host_srv_count", "dst_host_same_srv_rate", "dst_host_diff_srv_rate",
    "dst_host_same_src_port_rate", "dst_host_srv_diff_host_rate", "dst_host_serror_rate",
    "dst_host_srv_serror_rate", "dst_host_rerror_rate", "dst_host_srv_rerror_rate", "class",
]

INTRUSION_CATEGORICAL = [
    "protocol_type", "service", "flag", "land", "wrong_fragment", "urgent", "hot",
    "num_failed_logins", "logged_in", "num_compromised", "root_shell", "su_attempted",
    "num_root", "num_file_creations", "num_shells", "num_access_files", "num_outbound_cmds",
    "is_host_login", "is_guest_login", "class",
]

INTRUSION_NONNEGATIVE = ["dst_bytes", "src_bytes"]


@dataclasses.dataclass
class DatasetSpec:
    """Schema + run constants of one federated dataset.

    Fields mirror the reference CLI flags (`-name -datapath -selected_variables
    -categorical_list -nonnegative_list -date_dic -target_column -problem_type`) plus the
    literals the reference hard-codes: the per-epoch sample count 40000
    (`Server/dtds/distributed.py:583`) and the result-file stem 'Intrusion'
    (`Server/dtds/distributed.py:589, 679-684`).
    """

    name: str = "Intrusion"
    selected_variables: List[str] = dataclasses.field(default_factory=lambda: list(INTRUSION_COLUMNS))
    categorical_list: List[str] = dataclasses.field(default_factory=lambda: list(INTRUSION_CATEGORICAL))
    nonnegative_list: List[str] = dataclasses.field(default_factory=lambda: list(INTRUSION_NONNEGATIVE))
    date_dic: Dict[str, str] = dataclasses.field(default_factory=dict)
    target_column: str = "class"
    problem_type: str = "binary_classification"
    n_sample: int = 40000
    generator: Optional[str] = "intrusion"  # synthetic-data generator able to produce this schema

    def to_json(self) -> str:
        return json.dumps(dataclasses.asdict(self), indent=2)

    @classmethod
    def from_dict(cls, d: dict) -> "DatasetSpec":
        known = {f.name for f in dataclasses.fields(cls)}
        return cls(**{k: v for k, v in d.items() if k in known})

    @classmethod
    def from_json(cls, path: str) -> "DatasetSpec":
        with open(path) as f:
            return cls.from_dict(json.load(f))

    def copy(self) -> "DatasetSpec":
        return DatasetSpec.from_dict(json.loads(self.to_json()))


def intrusion_spec() -> DatasetSpec:
    return DatasetSpec()


def adult_spec() -> DatasetSpec:
    from .synthetic import ADULT_COLUMNS, ADULT_CATEGORICAL
    return DatasetSpec(name="Adult", selected_variables=list(ADULT_COLUMNS),
                       categorical_list=list(ADULT_CATEGORICAL), nonnegative_list=["capital-gain", "capital-loss"],
                       target_column="income", problem_type="binary_classification", generator="adult")


def covertype_spec() -> DatasetSpec:
    from .synthetic import covertype_columns
    cols, cats = covertype_columns()
    return DatasetSpec(name="Covertype", selected_variables=cols, categorical_list=cats, nonnegative_list=[],
                       target_column="Cover_Type", problem_type="multiclass_classification", generator="covertype")


def wide_spec(n_cols: int = 512, frac_categorical: float = 0.5) -> DatasetSpec:
    from .synthetic import wide_columns
    cols, cats = wide_columns(n_cols, frac_categorical)
    return DatasetSpec(name="Wide", selected_variables=cols, categorical_list=cats, nonnegative_list=[],
                       target_column=cats[-1], problem_type="multiclass_classification",
                       generator=f"wide:{n_cols}:{frac_categorical}")


BUILTIN_SPECS = {
    "intrusion": intrusion_spec,
    "adult": adult_spec,
    "covertype": covertype_spec,
    "wide": wide_spec,
}


def get_spec(name_or_path: str) -> DatasetSpec:
    key = name_or_path.lower()
    if key in BUILTIN_SPECS:
        return BUILTIN_SPECS[key]()
    return DatasetSpec.from_json(name_or_path)
