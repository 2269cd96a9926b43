"""CPU test of tools/pmc_extras.py: the marginal-step rule (PMC of --steps 2 minus --steps 1, per
kernel) on synthetic rocprofv3 counter CSVs, and the single-run fallback."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COLS = "Correlation_Id,Dispatch_Id,Agent_Id,Queue_Id,Process_Id,Thread_Id,Grid_Size,Kernel_Id,Kernel_Name," \
       "Workgroup_Size,LDS_Block_Size,Scratch_Size,VGPR_Count,Accum_VGPR_Count,SGPR_Count,Counter_Name,Counter_Value"


def write_pass(d, counter, rows):
    os.makedirs(os.path.join(d, counter, "box"), exist_ok=True)
    with open(os.path.join(d, counter, "box", "pmc_counter_collection.csv"), "w") as f:
        f.write(COLS + "\n")
        for i, (name, v) in enumerate(rows):
            f.write(f'{i},{i},1,1,1,1,256,{i},"{name}",256,0,0,64,0,32,{counter},{v}\n')


def run(src, tmp_path):
    out = tmp_path / "t.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_extras.py"), str(src), str(out), "t"],
                   check=True, capture_output=True)
    return json.loads(out.read_text())["workloads"]


def test_marginal_step_cancels_setup_and_check(tmp_path):
    d = tmp_path / "pmc" / "process"
    setup = [("void fill_splitmix_kernel(unsigned long*)", 4e6), ("__amd_rocclr_copyBuffer", 1e6)]
    check = [("__amd_rocclr_copyBuffer", 8e6)]                # parity copy-back after the run
    step = [("rs_code_kernel(int)", 3e6), ("void dm::leaf_kernel_quad<4>(int)", 5e6)]
    for k in (1, 2):
        write_pass(str(d / f"s{k}"), "FETCH_SIZE", setup + step * k + check)
        write_pass(str(d / f"s{k}"), "WRITE_SIZE", [(n, v / 2) for n, v in setup + step * k + check])
    w = run(tmp_path / "pmc", tmp_path)["process"]
    assert w["method"].startswith("marginal")
    assert set(w["kernels"]) == {"rs_code_kernel", "leaf_kernel_quad"}     # setup/check kernels cancel
    rs = w["kernels"]["rs_code_kernel"]
    assert rs["launches"] == 1 and rs["read_bytes"] == 3e6 * 2048 and rs["write_bytes"] == 1.5e6 * 1024
    assert w["traffic_bytes_per_step"] == (3e6 + 5e6) * 2048 + (1.5e6 + 2.5e6) * 1024
    assert w["setup_and_check_bytes"] == (4e6 + 1e6 + 8e6) * 2048 + (2e6 + 0.5e6 + 4e6) * 1024


def test_single_run_fallback_skips_setup_by_name(tmp_path):
    d = tmp_path / "pmc" / "plumbing"
    rows = [("void fill_splitmix_kernel(unsigned long*)", 4e6), ("at::native::zero_kernel", 1.0),
            ("void dm::leaf_kernel_quad<4>(int)", 5e6)]
    write_pass(str(d), "FETCH_SIZE", rows)
    write_pass(str(d), "WRITE_SIZE", rows)
    w = run(tmp_path / "pmc", tmp_path)["plumbing"]
    assert w["method"].startswith("single") and list(w["kernels"]) == ["leaf_kernel_quad"]
    assert w["traffic_bytes_per_step"] == 5e6 * 2048 + 5e6 * 1024
