"""tools/pmc_summary.py: the block-kernel step period of a PMC pass is found from the block-node
count up, so repeats inside a step (the 14x14 stage's identical bottlenecks) or a find step's
candidate launches ahead of the steps are not taken for a step."""
import csv
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _tool():
    spec = importlib.util.spec_from_file_location("pmc_summary", os.path.join(ROOT, "tools", "pmc_summary.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _write_pass(d, names, counters):
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "run_counter_collection.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, ["Dispatch_Id", "Kernel_Name", "Grid_Size", "VGPR_Count", "Accum_VGPR_Count",
                               "LDS_Block_Size", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for i, n in enumerate(names):
            for c, v in counters.items():
                w.writerow({"Dispatch_Id": i + 1, "Kernel_Name": n, "Grid_Size": 256, "VGPR_Count": 128,
                            "Accum_VGPR_Count": 0, "LDS_Block_Size": 0, "Counter_Name": c, "Counter_Value": v})


def test_step_period_skips_inner_repeats_and_find_step(tmp_path):
    t = _tool()
    assert t.min_launches() == 54  # ResNet-50 at 64 samples: 53 conv blocks + the classifier
    # a 55-launch step (one split-K block launches twice) whose tail repeats with period 3
    step = [f"k{i}" for i in range(25)] + ["a", "b", "c"] * 10
    find = [f"cand{i % 7}" for i in range(300)]
    names = find + step * 8
    _write_pass(str(tmp_path / "pass1"), names, {"FETCH_SIZE": 1.0})
    _write_pass(str(tmp_path / "pass2"), names, {"WRITE_SIZE": 2.0})
    out = t.summarise(str(tmp_path))
    assert out["launches_per_step"] == 55
    assert out["fetch_bytes_per_step"] == 55 * 1024 * 2
    assert out["write_bytes_per_step"] == 55 * 2 * 1024
