"""``python -m dtds.distributed`` — reference-compatible entry point (see :mod:`fed_tgan_amd.cli`)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from fed_tgan_amd.cli import main  # noqa: E402

if __name__ == "__main__":
    main(sys.argv[1:])
