"""Run a script with Python stack dumps every 30 s on stderr (diagnosing a stalled multi-rank
run): python scripts/ft_run.py bench.py --gpus 4 ...  (under torchrun as the training script)."""
import faulthandler
import runpy
import sys

faulthandler.dump_traceback_later(30, repeat=True)
sys.argv = sys.argv[1:]
runpy.run_path(sys.argv[0], run_name="__main__")
