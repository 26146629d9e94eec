"""Dev tool: host-side profile (cProfile) of bench.py --mode train steps."""
import cProfile
import pstats
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.argv = ["bench.py", "--mode", "train", "--steps", "30", "--warmup", "3"]
import bench  # noqa: E402

pr = cProfile.Profile()
pr.enable()
bench.main()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(35)
