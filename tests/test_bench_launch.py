"""bench.py's launcher logic (CPU): how `--gpus N` maps onto rank processes, without a GPU."""
import pytest

import bench


def test_single_process_default():
    assert bench.resolve_launch(1, {}) == ("rank", 1, 0, 0)


def test_gpus_n_without_launcher_spawns():
    assert bench.resolve_launch(8, {}) == ("spawn", 8)
    assert bench.resolve_launch(2, {"MASTER_ADDR": "127.0.0.1"}) == ("spawn", 2)


def test_torchrun_env_is_one_rank():
    env = {"WORLD_SIZE": "4", "RANK": "2", "LOCAL_RANK": "2"}
    assert bench.resolve_launch(4, env) == ("rank", 4, 2, 2)
    # `--gpus` left at its default under torchrun: the env decides
    assert bench.resolve_launch(1, env) == ("rank", 4, 2, 2)


def test_mismatched_world_refused():
    with pytest.raises(SystemExit):
        bench.resolve_launch(8, {"WORLD_SIZE": "4", "RANK": "0", "LOCAL_RANK": "0"})
    with pytest.raises(SystemExit):
        bench.resolve_launch(0, {})


def test_spawned_rank_env_round_trips():
    for r in range(3):
        env = bench.rank_env(r, 3, 29555)
        assert env["MASTER_ADDR"] == "127.0.0.1" and env["MASTER_PORT"] == "29555"
        assert bench.resolve_launch(3, env) == ("rank", 3, r, r)


def test_host_cores_reports_affinity():
    import os
    n, quota, model = bench.host_cores()
    assert n == len(os.sched_getaffinity(0)) and isinstance(model, str)
    assert quota is None or quota > 0
