"""Column-kind tags shared by the data and feature layers.

Parity: `Server/dtds/data/constants.py:1-3` (CATEGORICAL / CONTINUOUS / ORDINAL) and
the client's extra BIMODAL tag (`Client/.../dtds/data/constants.py:4`).

The on-disk meta JSON written by the reference spells the continuous kind
"continous" (`Server/dtds/data/utils/file_generator.py:206`); we keep that exact
spelling in files we write so downstream tooling that reads them keeps working.
"""

CATEGORICAL = "categorical"
CONTINUOUS = "continuous"
ORDINAL = "ordinal"
BIMODAL = "bimodal"

# spelling used inside the meta JSON files (reference quirk, kept for output-compat)
META_CONTINUOUS = "continous"

# literal used by the reference pipeline for missing cells before/after decoding
EMPTY = "empty"
