"""World-size-2 and -8 (gloo, CPU) coverage of the multi-GPU path (SURVEY.md 8e;
world size 8 rehearses the driver's 8-GPU launch: 8 ranks, one shard each).

The path shards with no data-path collective: each rank owns a contiguous
range of blocks (weak scaling, bench.py) or a byte-balanced range of spans
(hcrc_batch_multi).  These tests run the same sharding helpers bench.py uses
(wipdb_amd.shard) in two gloo processes; each rank computes its shard with
the library's host entry point (hcrc_cpu_batch -- the GPU kernel needs a
device), and the union is checked against the oracle.  The all_gather below
is the test's checker, not part of the path; the only collective the bench
itself issues is the MAX-over-ranks timing reduction, exercised here too.
"""
import os
import socket

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SEED = 0x4B10C5
BLOCK = 4096


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _mixed_spans(seed: int, nbytes: int):
    rng = np.random.default_rng(seed)
    buckets = np.array([512, 1024, 2048, 4096, 8192, 16384, 32768, 65536])
    p = 1.0 / np.arange(1, 9) ** 0.99
    p /= p.sum()
    offs, lens, cur = [], [], 3
    while True:
        L = int(rng.choice(buckets, p=p))
        n = L + int(rng.integers(0, L // 8 + 1))
        if cur + n + 5 > nbytes:
            break
        offs.append(cur)
        lens.append(n)
        cur += n + 5
    return np.array(offs, np.uint64), np.array(lens, np.uint32)


def _worker(rank: int, world: int, port: int, blocks: int, outdir: str):
    import sys
    sys.path.insert(0, REPO)
    import torch
    import torch.distributed as dist
    from tests.golden.common import splitmix64_bytes
    from wipdb_amd import cpu_batch
    from wipdb_amd.shard import block_shard, byte_balanced_cuts, max_over_ranks

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        # (1) weak-scaling block shards, data regenerated per rank from the seed
        first, n = block_shard(rank, world, blocks)
        buf = splitmix64_bytes(SEED, n * BLOCK, start=first * BLOCK)
        crc = cpu_batch(buf, np.arange(n, dtype=np.uint64) * BLOCK, np.full(n, BLOCK, np.uint32))
        t = torch.from_numpy(crc.view(np.int32).copy())
        parts = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(parts, t)  # checker only
        # (2) byte-balanced span shards over one shared SST-like buffer
        sbuf = splitmix64_bytes(SEED ^ 0x55, 3 << 20)
        offs, lens = _mixed_spans(7, sbuf.size)
        cut = byte_balanced_cuts(lens, world)
        lo, hi = cut[rank], cut[rank + 1]
        scrc = cpu_batch(sbuf, offs[lo:hi], lens[lo:hi], mask_output=True)
        sparts = [None] * world
        dist.all_gather_object(sparts, (lo, hi, scrc))  # checker only
        # (3) the bench's timing reduction
        tmax = max_over_ranks(float(rank + 1))
        if rank == 0:
            np.save(os.path.join(outdir, "blocks.npy"),
                    np.concatenate([p.numpy() for p in parts]).view(np.uint32))
            got = np.zeros(lens.size, np.uint32)
            covered = np.zeros(lens.size, np.int32)
            for a, b, c in sparts:
                got[a:b] = c
                covered[a:b] += 1
            np.save(os.path.join(outdir, "spans.npy"), got)
            np.save(os.path.join(outdir, "covered.npy"), covered)
            with open(os.path.join(outdir, "tmax.txt"), "w") as f:
                f.write(repr(tmax))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(400)
@pytest.mark.parametrize("world", [2, 8])
def test_gloo_world_shards(tmp_path, oracle, world):
    import torch.multiprocessing as mp
    from tests.golden.common import splitmix64_bytes
    blocks = 96
    mp.spawn(_worker, args=(world, _free_port(), blocks, str(tmp_path)), nprocs=world, join=True)
    got = np.load(tmp_path / "blocks.npy")
    full = splitmix64_bytes(SEED, world * blocks * BLOCK)
    n = world * blocks
    want = oracle.batch(full, np.arange(n, dtype=np.uint64) * BLOCK, np.full(n, BLOCK, np.uint32))
    np.testing.assert_array_equal(got, want)

    sbuf = splitmix64_bytes(SEED ^ 0x55, 3 << 20)
    offs, lens = _mixed_spans(7, sbuf.size)
    assert (np.load(tmp_path / "covered.npy") == 1).all()  # disjoint and complete
    np.testing.assert_array_equal(np.load(tmp_path / "spans.npy"),
                                  oracle.batch(sbuf, offs, lens, mask=True))
    assert float((tmp_path / "tmax.txt").read_text()) == float(world)


def test_byte_balanced_cuts_match_cpp_rule():
    from wipdb_amd.shard import byte_balanced_cuts

    def cpp(lengths, ndev):  # restatement of hcrc_batch_multi's loop
        count = len(lengths)
        total = sum(int(v) + 64 for v in lengths)
        cut = [count] * (ndev + 1)
        cut[0], acc, d = 0, 0, 1
        for i in range(count):
            if d >= ndev:
                break
            acc += int(lengths[i]) + 64
            while d < ndev and acc >= total * d // ndev:
                cut[d] = i + 1
                d += 1
        return cut

    rng = np.random.default_rng(0)
    for _ in range(500):
        n, ndev = int(rng.integers(0, 40)), int(rng.integers(1, 9))
        lens = rng.integers(0, 70000, n)
        if rng.random() < 0.3:
            lens[:] = int(rng.integers(0, 3))
        assert byte_balanced_cuts(lens, ndev) == cpp(lens, ndev)
    # balance on a Zipf SST-like mix: every shard within one max span of ideal
    _, lens = _mixed_spans(3, 64 << 20)
    cut = byte_balanced_cuts(lens, 8)
    w = lens.astype(np.int64) + 64
    shares = [int(w[cut[k]:cut[k + 1]].sum()) for k in range(8)]
    assert max(shares) - min(shares) <= 2 * int(w.max())


def test_block_shard_weak():
    from wipdb_amd.shard import block_shard
    assert block_shard(0, 8, 1 << 20) == (0, 1 << 20)
    assert block_shard(7, 8, 1 << 20) == (7 << 20, 1 << 20)
    with pytest.raises(ValueError):
        block_shard(8, 8, 10)
