"""A/B a rollout-kernel build: python tools/_ablib.py build/libX.so [B]"""
import json, os, subprocess, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import citadels_self_play_amd._lib as LL
LL.LIB_PATH = sys.argv[1]
sys.argv = ["bench.py", "--no-cpu-baseline", "--no-pmc", "--no-cfr", "--steps", "10"] + (["--streams", os.environ["AB_STREAMS"]] if os.environ.get("AB_STREAMS") else []) + (["--batch", sys.argv[2]] if len(sys.argv) > 2 else []) + os.environ.get("AB_ARGS", "").split()
import bench
bench.main()
