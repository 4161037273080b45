"""Multi-rank path on CPU (gloo, world_size 2 and 3): replicate sharding + all-gather must give
exactly the rows and statistics of a single-process run (replicate results are a pure function
of the replicate id, as they are on the GPU engine)."""
import os
import socket

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class StubPrepared:
    """Row producer with the PreparedRun protocol; row r depends only on replicate id r."""

    row_len = 7

    def boot(self, first, n):
        rows = np.empty((n, self.row_len))
        ok = np.ones(n, dtype=np.uint8)
        for i in range(n):
            rng = np.random.default_rng(1000 + first + i)
            rows[i] = rng.normal(size=self.row_len)
            ok[i] = 0 if (first + i) % 11 == 5 else 1
        return rows, ok


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_reps, outdir):
    import sys

    sys.path.insert(0, ROOT)
    import importlib

    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    D = importlib.import_module("oaxaca-blinder-rs_amd.distributed")
    rows, ok = D.gather_rows(StubPrepared(), n_reps)
    np.savez(os.path.join(outdir, f"r{rank}.npz"), rows=rows, ok=ok)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n_reps", [(2, 37), (3, 10), (2, 1)])
def test_gather_equals_single_process(tmp_path, world, n_reps):
    import torch.multiprocessing as mp

    mp.start_processes(_worker, args=(world, _free_port(), n_reps, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    ref_rows, ref_ok = StubPrepared().boot(0, n_reps)
    for r in range(world):
        z = np.load(tmp_path / f"r{r}.npz")
        assert np.array_equal(z["rows"], ref_rows)
        assert np.array_equal(z["ok"], ref_ok)


def test_shard_ranges():
    import importlib
    import sys

    sys.path.insert(0, ROOT)
    D = importlib.import_module("oaxaca-blinder-rs_amd.distributed")
    for n in (0, 1, 7, 10000, 10001):
        for w in (1, 2, 3, 8):
            cover = []
            for r in range(w):
                first, count, per = D.shard(n, r, w)
                assert count <= per
                cover += list(range(first, first + count))
            assert cover == list(range(n))
