"""The in-process leg launched the way rank 0 launches it (run_child_leg: own session, rank env stripped),
from a plain process with no ranks alive: does the launch path itself change the host feed?"""
import json, os, sys
sys.path.insert(0, os.getcwd())
import bench
r, hung = bench.run_child_leg([sys.executable, os.path.abspath("bench.py"), "--workload", "inprocess", "--gpus", "1",
                               "--inproc-gib", "16", "--same-device", "--inproc-devices", "8"], "in_process", 300)
print(json.dumps({"hung": hung, "host_feed": r.get("host_feed")}))
