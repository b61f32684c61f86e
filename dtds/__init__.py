"""Compatibility package: ``python -m dtds.distributed`` runs the fed_tgan_amd federation with the
reference's command-line surface (`Server/dtds/distributed.py:894-971`)."""
