"""`import wespeaker` drop-in (wespeaker/__init__.py:1-2 exports load_model,
load_model_pt): the same names from wespeaker_hubert_amd.  A recipe directory
whose `wespeaker` symlink (examples/*/v2/wespeaker -> ../../../wespeaker) is
re-pointed at <repo>/compat/wespeaker runs unchanged on this package."""
import os
import sys

_REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.realpath(__file__))))
if _REPO not in sys.path:
    sys.path.insert(0, _REPO)

from wespeaker_hubert_amd import load_model, load_model_pt  # noqa: E402,F401
