"""bench.py's cpu_baseline leg (CPU): the oracle timed on one thread and on every host
thread, threads stepping independent batches through ctypes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def test_cpu_baseline_reports_thread_count():
    import bench
    from mapf_amd.maps import generate_warehouse
    line = bench.cpu_baseline(generate_warehouse(10, 10), 10, 10, 4, 11, 6, 1.0)
    assert line["kind"] == "port" and line["unit"] == "agent-steps/s"
    assert line["cores"] == bench.host_threads() >= 1
    assert line["value"] > 0 and line["single_thread_value"] > 0
    assert abs(line["per_core_value"] * line["cores"] - line["value"]) < 1.0 + 1e-6 * line["value"]
    assert f"{line['cores']} threads" in line["sample"] and "nproc" in line["host"]


def test_host_threads_is_the_gpu_share(monkeypatch):
    """On the GPU box OMP_NUM_THREADS names this GPU's CPU share (16): the baseline runs that
    many threads, not nproc."""
    import bench
    monkeypatch.setenv("OMP_NUM_THREADS", "3")
    assert bench.host_threads() == min(3, len(os.sched_getaffinity(0)))
    monkeypatch.delenv("OMP_NUM_THREADS")
    assert bench.host_threads() == len(os.sched_getaffinity(0))


def test_roofline_bytes_match_design():
    """3,001.25 B per agent-step for the rollout / step_observe kernels at c2;
    SURVEY.md §8d's observe formula at c5 (3,424.6 B) + the BFS channel's map reads
    (F*F*2 + 2 = 244 B) = 3,668.6 B; the rollout kernels' at c5 3,728.5 B."""
    import bench
    assert bench.fused_bytes_per_agent(6, 11, 20, 20, 8) == 3001.25
    assert abs(bench.observe_bytes_per_agent(7, 11, 80, 80, 64) - 3668.6) < 0.1
    assert abs(bench.fused_bytes_per_agent(7, 11, 80, 80, 64) - 3728.5) < 0.1


def test_threaded_batches_match_single_thread():
    """Threads share nothing: a batch stepped alongside others ends where it ends alone
    (oc_batch_run leaves the last env's observation in the batch's buffers)."""
    import threading

    from mapf_amd.maps import generate_warehouse
    from oracle import oracle as O
    world = generate_warehouse(20, 20)
    cfg = O.make_config(20, 20, 8, 11, 6, human_mode=1, goal_mode=1, fix_choice=1, seed=99)
    alone = O.OracleBatch(cfg, world, 4)
    want = [alone.run(7) for _ in range(3)], alone.obs.copy(), alone.vec.copy()
    batches = [O.OracleBatch(cfg, world, 4) for _ in range(4)]
    got = [None] * 4

    def work(i):
        got[i] = [batches[i].run(7) for _ in range(3)]

    ts = [threading.Thread(target=work, args=(i,)) for i in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for i, b in enumerate(batches):
        assert got[i] == want[0]
        assert (b.obs == want[1]).all() and (b.vec == want[2]).all()


def test_all_cores_figure_is_labelled():
    """`value` is this GPU's CPU share, labelled as such; the all-host-cores
    figure is reported beside it (per-thread rate x nproc, named an extrapolation)."""
    import bench
    from mapf_amd.maps import generate_warehouse
    line = bench.cpu_baseline(generate_warehouse(10, 10), 10, 10, 4, 11, 6, 0.5)
    assert line["value_label"].startswith(f"{line['cores']} of {line['host_cores']} host cores")
    assert abs(line["all_host_cores_value"] - line["per_core_value"] * line["host_cores"]) <= 1.0 + 1e-6 * line["value"]
    assert "extrapolated" in line["all_host_cores_basis"]


def test_gpus_flag_launches_that_many_ranks(monkeypatch):
    """`bench.py --gpus N` with no launcher around it starts N ranks of the same
    command under torch.distributed.run (a child process; 127.0.0.1 rendezvous) and exits with its
    code -- before anything touches the GPU."""
    import subprocess
    import bench
    seen = {}

    def fake_call(cmd, env=None):
        seen["cmd"], seen["env"] = cmd, env
        return 7
    monkeypatch.setattr(subprocess, "call", fake_call)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "3"])
    try:
        bench.main()
        raise AssertionError("main() returned")
    except SystemExit as e:
        assert e.code == 7
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--master-addr=127.0.0.1" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"] and cmd[-5].endswith("bench.py")
