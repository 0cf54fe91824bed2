"""Recipe launcher for wespeaker/bin/compute_det.py: runs wespeaker_hubert_amd.bin.compute_det
with the same command line (see compat/wespeaker/__init__.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.realpath(__file__)))
from _launch import run  # noqa: E402

run("wespeaker_hubert_amd.bin.compute_det")
