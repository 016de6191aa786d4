"""Runs scripts/tci2_configs.py's named configs with the process map saved by the package's exit
hook (TCI_EXIT_DIAG, tci_amd/_lib.py), so frames of an exit-time fault (e.g. under rocprofv3) can
be resolved to libraries.

  python scripts/exit_diag.py <maps-out> [tci2 config names...]
"""
import os
import runpy
import sys

os.environ["TCI_EXIT_DIAG"] = os.path.abspath(sys.argv[1])
script = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tci2_configs.py")
sys.argv = [script] + sys.argv[2:]
runpy.run_path(script, run_name="__main__")
