#!/usr/bin/env python3
"""cProfile of tools/bench_constopt.py's workload (host vs engine time)."""
import cProfile
import pstats
import runpy
import sys
from pathlib import Path

sys.argv = [str(Path(__file__).with_name("bench_constopt.py"))] + sys.argv[1:]
pr = cProfile.Profile()
pr.enable()
runpy.run_path(sys.argv[0], run_name="__main__")
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(15)
