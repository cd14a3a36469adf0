"""cProfile of bench.py with the autograd engine on the calling thread (so the Python backward
functions show up in the profile).  Usage: python tools/host_prof.py OUT.prof [bench.py args]"""
import cProfile
import os
import sys

import torch

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
torch.autograd.set_multithreading_enabled(False)
out = sys.argv[1]
sys.argv = ["bench.py"] + sys.argv[2:]
import bench  # noqa: E402

cProfile.run("bench.main()", out)
