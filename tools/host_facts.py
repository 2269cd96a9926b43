"""Print the host facts bench.py's cpu_baseline reports (CPU model, counts, affinity, cgroup quota)."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import host_cpu_facts
print(json.dumps(host_cpu_facts(), indent=1))
