"""Shared by the recipe launchers in this directory: run a wespeaker_hubert_amd.bin
module as __main__ with the caller's argv (the reference scripts' flags are
accepted unchanged; each module cites the reference script it replaces)."""
import os
import runpy
import sys


def run(module: str) -> None:
    repo = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.realpath(__file__)))))
    if repo not in sys.path:
        sys.path.insert(0, repo)
    runpy.run_module(module, run_name="__main__", alter_sys=True)
