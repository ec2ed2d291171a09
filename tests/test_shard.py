"""Multi-rank sharding + result all-gather (gloo, world_size 2 and 3).

On CPU the per-shard verifier is injected: the CPU oracle stands in for the
gfx950 kernel so the distributed plumbing (shard bounds, padding, gather order)
is tested without a GPU.  The -m gpu tests run the same function with the HIP
kernel per shard (gloo world of 2 on the box's GPU) and the RCCL gather branch.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_range_covers_exactly():
    from ouroboros_network_amd.shard import shard_range

    for n in (0, 1, 7, 64, 1000, 1 << 20):
        for world in (1, 2, 3, 8):
            spans = [shard_range(n, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            for (a, b), (c, _) in zip(spans, spans[1:]):
                assert b == c and a <= b


def test_bench_step_shards_is_configs3_strong_by_default():
    """bench.py --gpus N > 1 measures configs[3] as written: ONE batch of
    1,048,576 headers per step cut into N/G contiguous shards (SURVEY.md
    §8(d)); --weak keeps 1,048,576 per GPU; N = 1 is the plain 1M batch."""
    import bench

    for world in (2, 4, 8):
        spans = [bench.step_shards(world, r, 1 << 20, -1, False) for r in range(world)]
        assert all(s[0] for s in spans)                       # strong
        assert all(s[3] == 1 << 20 for s in spans)            # global batch
        assert [s[1] for s in spans] == [(1 << 20) // world] * world
        assert [s[2] for s in spans] == [r * (1 << 20) // world for r in range(world)]
        weak = [bench.step_shards(world, r, 1 << 20, -1, True) for r in range(world)]
        assert all(not s[0] and s[1] == 1 << 20 and s[3] == world << 20 for s in weak)
        assert [s[2] for s in weak] == [r << 20 for r in range(world)]
    assert bench.step_shards(1, 0, 1 << 20, -1, False) == (False, 1 << 20, 0, 1 << 20)
    # an explicit global batch that does not divide evenly: ceil(N/G), contiguous
    spans = [bench.step_shards(3, r, 0, 1000, False) for r in range(3)]
    assert [(s[1], s[2]) for s in spans] == [(334, 0), (334, 334), (332, 668)]


def _worker(rank, world, port, out_dir, use_gpu=False):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "tests"))
    import json

    import torch.distributed as dist

    import oracle_ffi as O
    from ouroboros_network_amd import header as H
    from ouroboros_network_amd.shard import verify_sharded

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    kats = json.load(open(os.path.join(root, "tests", "golden", "reference_kats.json")))
    hs = kats["headers"] * 2
    parsed = [H.parse_header(bytes.fromhex(h["raw"])) for h in hs]
    ea = [bytes.fromhex(h["eta_alpha"]) for h in hs]
    la = [bytes.fromhex(h["leader_alpha"]) for h in hs]
    la[3] = bytes(32)  # one leader VRF fails
    batch = H.pack(parsed, ea, la, slots_per_kes_period=100)
    if use_gpu:  # the gfx950 kernel per shard (every rank on GPU 0 of the box)
        import torch

        torch.cuda.set_device(0)
        v, be, bl = verify_sharded(batch)
    else:
        v, be, bl = verify_sharded(batch, verify=lambda b: O.tpraos_verify_batch(b, threads=1))
    np.save(os.path.join(out_dir, f"v{rank}.npy"), v)
    np.save(os.path.join(out_dir, f"be{rank}.npy"), be)
    np.save(os.path.join(out_dir, f"bl{rank}.npy"), bl)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_verify_sharded_gloo(tmp_path, world, kats):
    import oracle_ffi as O
    from ouroboros_network_amd import header as H

    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    hs = kats["headers"] * 2
    parsed = [H.parse_header(bytes.fromhex(h["raw"])) for h in hs]
    ea = [bytes.fromhex(h["eta_alpha"]) for h in hs]
    la = [bytes.fromhex(h["leader_alpha"]) for h in hs]
    la[3] = bytes(32)
    want = O.tpraos_verify_batch(H.pack(parsed, ea, la, slots_per_kes_period=100))
    for r in range(world):
        np.testing.assert_array_equal(np.load(tmp_path / f"v{r}.npy"), want[0])
        np.testing.assert_array_equal(np.load(tmp_path / f"be{r}.npy"), want[1])
        np.testing.assert_array_equal(np.load(tmp_path / f"bl{r}.npy"), want[2])
    assert want[0][3] & 0x0F == 0x07 and (np.delete(want[0], 3) & 0x0F == 0x0F).all()


@pytest.mark.gpu
def test_verify_sharded_hip_per_shard_gloo(tmp_path, kats):
    """shard.verify_sharded with the REAL per-shard verifier (the HIP kernel
    through the C ABI, both ranks on the box's one GPU) over a gloo world of 2:
    every rank's gathered results equal the oracle over the whole batch."""
    import oracle_ffi as O
    from ouroboros_network_amd import header as H

    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), True), nprocs=world, join=True)
    hs = kats["headers"] * 2
    parsed = [H.parse_header(bytes.fromhex(h["raw"])) for h in hs]
    ea = [bytes.fromhex(h["eta_alpha"]) for h in hs]
    la = [bytes.fromhex(h["leader_alpha"]) for h in hs]
    la[3] = bytes(32)
    want = O.tpraos_verify_batch(H.pack(parsed, ea, la, slots_per_kes_period=100))
    for r in range(world):
        np.testing.assert_array_equal(np.load(tmp_path / f"v{r}.npy"), want[0])
        np.testing.assert_array_equal(np.load(tmp_path / f"be{r}.npy"), want[1])
        np.testing.assert_array_equal(np.load(tmp_path / f"bl{r}.npy"), want[2])


def _nccl_worker(rank, world, port, out_dir):
    import torch
    import torch.distributed as dist

    from ouroboros_network_amd.shard import all_gather_results, pack_results

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      HSA_ENABLE_IPC_MODE_LEGACY="0")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    n = 1000
    g = torch.Generator().manual_seed(3)
    v = torch.randint(0, 16, (n,), generator=g, dtype=torch.uint8).to(dev)
    be = torch.randint(0, 256, (n * 64,), generator=g, dtype=torch.uint8).to(dev)
    bl = torch.randint(0, 256, (n * 64,), generator=g, dtype=torch.uint8).to(dev)
    full = all_gather_results(pack_results(v, be, bl), n, world)
    torch.cuda.synchronize()
    ok = bool(torch.equal(full.cpu(), pack_results(v, be, bl).cpu()))
    dist.destroy_process_group()
    with open(os.path.join(out_dir, "ok"), "w") as f:
        f.write("1" if ok else "0")


@pytest.mark.gpu
def test_result_gather_over_rccl(tmp_path):
    """The device branch of all_gather_results (one flat RCCL all-gather into
    the result tensor) on a one-rank nccl group: the only multi-rank
    collective bench.py uses at N > 1, exercised on the one-GPU box."""
    mp.spawn(_nccl_worker, args=(1, _free_port(), str(tmp_path)), nprocs=1, join=True)
    assert (tmp_path / "ok").read_text() == "1"


def _topology_worker(rank, world, port, out_dir, shared):
    import json
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import torch.distributed as dist

    from ouroboros_network_amd.shard import check_rank_devices

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    info = {"rank": rank, "device": 0 if shared else rank,
            "bus_id": "0000:05:00.0" if shared else f"0000:{5 + rank:02x}:00.0"}
    infos = [None] * world
    dist.all_gather_object(infos, info)
    res = {}
    for name, kw in (("exact", dict(expected_world=world)),
                     ("wrong_n", dict(expected_world=world + 1)),
                     ("shared_ok", dict(expected_world=world, allow_shared=True))):
        try:
            check_rank_devices(infos, **kw)
            res[name] = "ok"
        except RuntimeError as e:
            res[name] = str(e)
    dist.destroy_process_group()
    with open(os.path.join(out_dir, f"r{rank}.json"), "w") as f:
        json.dump(res, f)


def test_rank_devices_across_nodes():
    """two nodes have the same PCI bus ids and local indices; a
    world spanning them is valid (a GPU is (host, bus id)), while two ranks
    on one host and one bus id still share a GPU."""
    from ouroboros_network_amd.shard import check_rank_devices

    two_nodes = [{"rank": r, "device": r % 2, "bus_id": f"0000:{5 + r % 2:02x}:00.0",
                  "host": f"node{r // 2}"} for r in range(4)]
    check_rank_devices(two_nodes, 4)
    no_bus = [{"rank": r, "device": 0, "bus_id": None, "host": f"node{r}"} for r in range(2)]
    check_rank_devices(no_bus, 2)
    same = [dict(two_nodes[0]), dict(two_nodes[1]), dict(two_nodes[2]), dict(two_nodes[3])]
    same[2]["host"] = "node0"
    with pytest.raises(RuntimeError, match="share GPUs"):
        check_rank_devices(same, 4)


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("shared", [False, True])
def test_bench_rank_device_checks_gloo(tmp_path, world, shared):
    """bench.py --gpus N refuses a line unless the process group has N ranks
    and (outside the gloo rehearsal) every rank drives its own GPU: the check
    run over a real gloo world of 2 and 3 ranks with distinct and with shared
    devices."""
    import json

    mp.spawn(_topology_worker, args=(world, _free_port(), str(tmp_path), shared), nprocs=world,
             join=True)
    for r in range(world):
        res = json.load(open(tmp_path / f"r{r}.json"))
        assert res["wrong_n"].startswith("world size")
        assert res["shared_ok"] == "ok"
        if shared:
            assert "share GPUs" in res["exact"]
        else:
            assert res["exact"] == "ok"
