"""bench.py's host-side pieces that need no GPU: the CPU baseline (the reference's
fp32 CPU forward at a given batch, 1 warm-up + timed iterations, CPU model recorded) and the
int8-fused floors it reports beside the roofline."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def test_cpu_baseline_shape_and_fields():
    import bench
    r = bench.cpu_baseline("resnet18", "r18_u8", 2, iters=1)
    assert r["unit"] == "images/s" and r["kind"] == "port" and r["value"] > 0
    assert r["cores"] >= 1 and r["cpu_model"] and "batch 2" in r["sample"] and "1 warm-up" in r["sample"]


def test_int8_fused_floors_match_baseline_md():
    import bench
    # BASELINE.md 3, int8-fused bound column
    assert bench.INT8_FUSED_FLOOR_MS == {"r50_mixed": (256, 0.666), "r18_u8": (256, 0.179), "r34_4bit": (512, 0.742)}
    assert set(bench.INT8_FUSED_FLOOR_MS) == set(bench.CONFIGS)
