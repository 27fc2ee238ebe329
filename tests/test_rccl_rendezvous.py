"""RCCL unique-id rendezvous without GPUs (csrc/engine/rccl.cpp rendezvous_id).

The first multi-GPU run must not be able to hand a communicator a stale or a
foreign id. Three gloo ranks drive the exact store protocol of Rccl's
constructor with fake ids: two world communicators in a row plus a
MPI_Comm_split-style {0,1} / {2} split (reference oink/universe.cpp:55-88),
and the Python Comm.split path that OINK -partition uses.
"""
import os

from test_distributed_cpu import run_world


def case_rendezvous(comm):
    import torch.distributed as dist
    from gpu_mapreduce_amd._ext import C
    store = dist.distributed_c10d._get_default_store()
    r = comm.rank
    got = {}
    # two world communicators, created in the same order on every rank
    got["world0"] = C.rccl_rendezvous_probe(store, "world", [0, 1, 2], r)
    got["world1"] = C.rccl_rendezvous_probe(store, "world", [0, 1, 2], r)
    # split {0,1} / {2}: only the pair needs an id ({2} is a one-rank comm)
    if r in (0, 1):
        got["pair"] = C.rccl_rendezvous_probe(store, "split", [0, 1], r)
    # a second split with the same member list but a different creation
    got["pair2"] = C.rccl_rendezvous_probe(store, "split", [0, 1], r) if r in (0, 1) else None
    dist.barrier()
    # rank 0 deleted every key after all members acknowledged
    leftover = [k for v in got.values() if v for k in (v[0], v[0] + "/ack") if store.check([k])]
    return {k: (v[0], bytes(v[1])) if v else None for k, v in got.items()}, leftover


def test_rendezvous_keys_are_unique_and_ids_match():
    out = run_world("test_rccl_rendezvous:case_rendezvous", 3)
    per = {r: out[r][0] for r in range(3)}
    for r in range(3):
        assert out[r][1] == [], f"rank {r} sees undeleted id keys {out[r][1]}"
    # every member of a communicator fetched the id rank 0 published, under one key
    for name, ranks in (("world0", [0, 1, 2]), ("world1", [0, 1, 2]), ("pair", [0, 1]), ("pair2", [0, 1])):
        keys = {per[r][name][0] for r in ranks}
        ids = {per[r][name][1] for r in ranks}
        assert len(keys) == 1 and len(ids) == 1, (name, keys)
        assert len(next(iter(ids))) == 128
    # no two communicators share a key or an id
    keys = [per[0][n][0] for n in ("world0", "world1", "pair", "pair2")]
    ids = [per[0][n][1] for n in ("world0", "world1", "pair", "pair2")]
    assert len(set(keys)) == 4 and len(set(ids)) == 4, keys
    assert "pair" not in per[2] or per[2]["pair2"] is None


def case_python_split(comm):
    """Comm.split (OINK -partition): natives over distinct member lists,
    world-rank monitor, and one native communicator per member set."""
    sub = comm.split(0 if comm.rank < 2 else 1)
    n1 = comm.native
    n2 = type(comm)(comm.group, device=comm.device).native   # a second Comm over the world
    return {"members": list(sub.members), "native_members": list(sub.native.members),
            "sub_size": sub.native.size, "same_world_native": n1 is n2,
            "sum": sub.allreduce(comm.rank + 1), "world_members": list(n1.members),
            "info": dict(n1.rccl_info())}


def test_python_split_members_and_shared_native():
    out = run_world("test_rccl_rendezvous:case_python_split", 3)
    assert out[0]["members"] == out[1]["members"] == [0, 1]
    assert out[2]["members"] == [2]
    assert out[0]["native_members"] == [0, 1] and out[0]["sub_size"] == 2
    assert out[0]["sum"] == out[1]["sum"] == 3 and out[2]["sum"] == 3
    for r in range(3):
        assert out[r]["same_world_native"], "a second Comm over the same ranks must share the native communicator"
        assert out[r]["world_members"] == [0, 1, 2]
        # CPU engine: no RCCL communicator in this process
        assert out[r]["info"]["comm_count"] == -1 and out[r]["info"]["live_comms"] == 0


def case_native_split(comm):
    """the native Comm::split (OINK's C++ -partition path) over the store transport"""
    from gpu_mapreduce_amd._ext import C
    n = comm.native
    return list(n.members), n.allreduce([comm.rank], 0)


def test_native_members_world():
    out = run_world("test_rccl_rendezvous:case_native_split", 3)
    for r in range(3):
        assert out[r] == ([0, 1, 2], [3])
