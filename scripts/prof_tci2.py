"""cProfile one TCI2 config (scripts/tci2_configs.py name) after a warm-up run."""
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import tci2_configs as C  # noqa: E402

name = sys.argv[1]
cs = C.configs()
cs[name]()
cProfile.run(f"cs[{name!r}]()", "/tmp/prof.out")
pstats.Stats("/tmp/prof.out").sort_stats("tottime").print_stats(int(sys.argv[2]) if len(sys.argv) > 2 else 20)
