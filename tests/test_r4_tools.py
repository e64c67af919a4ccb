"""Round-4 helper tools on CPU: the stream-timeline overlap accounting (tools/stream_timeline.py),
the MFMA-busy formula (tools/pmc_table.py) and the collective flight recorder (parallel/comm.py)."""
import csv
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def test_stream_timeline_accounting(tmp_path, capsys):
    import json

    import stream_timeline

    rows = [  # (name, start, end, stream); times in ns
        ("adamw_kernel", 0, 10, 0),
        ("gemm", 100, 1100, 1), ("nxd::diag::cu_stream_kernel", 600, 1600, 3), ("copy", 1600, 1700, 3),
        ("nxd::fab::bwd_kernel", 1800, 2800, 2), ("nxd::diag::cu_stream_kernel", 2000, 2300, 3),
        ("adamw_kernel", 3000, 3010, 0),
    ]
    p = tmp_path / "t.csv"
    with open(p, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp", "Stream_Id"])
        for n, a, b, q in rows:
            w.writerow([n, a * 10000, b * 10000, q])   # 1 unit = 10 us
    stream_timeline.main(str(p), as_json=True)
    rec = json.loads(capsys.readouterr().out)
    st = rec["step"]
    # (one AdamW group: the whole trace is the step) compute = 2 x adam (10) + gemm [100,1100] +
    # fab [1800,2800]; link = [600,1700] + [2000,2300]
    assert st["compute_ms"] == 20.2 and st["link_ms"] == 14.0
    assert st["overlap_ms"] == 8.0            # [600,1100] + [2000,2300]
    assert st["exposed_link_ms"] == 6.0       # [1100,1700]


def test_mfma_busy_fraction():
    from pmc_table import mfma_busy_fraction

    # a dispatch of 1e6 cycles on all 1024 SIMDs with every SIMD busy half the time
    assert abs(mfma_busy_fraction(0.5 * 1024 * 1e6, 8 * 1e6) - 0.5) < 1e-12


def test_flight_recorder_records_collectives():
    from neuronx_distributed_llama3_2_amd.parallel import comm

    if not dist.is_initialized():
        dist.init_process_group("gloo", rank=0, world_size=1, init_method="tcp://127.0.0.1:29547")
    try:
        t = torch.ones(3)
        comm.all_reduce(t)
        o = torch.empty(3)
        comm.all_gather_into_tensor(o, t)
        last = comm.flight_record(2)
        assert last[0].split(" ", 1)[1].startswith("all_reduce(3,) float32 ws=1")
        assert "all_gather(3,)" in last[1]
        n0, n1 = int(last[0].split()[0][1:]), int(last[1].split()[0][1:])
        assert n1 == n0 + 1
    finally:
        dist.destroy_process_group()
