"""Checkpoint / restart of MR data (save/load of device KV and KMV), the
host spill tier, and the stats/timer outputs."""
import pytest
import torch

import gpu_mapreduce_amd as g


def _fill(mr):
    def gen(i, kv):
        for j in range(200):
            kv.add(f"w{(i * 31 + j) % 17}", j * 1.5)
    mr.map(4, gen)


@pytest.mark.parametrize("dev", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_save_load_kv_kmv(tmp_path, dev):
    mr = g.MapReduce(device=dev)
    _fill(mr)
    mr.save(tmp_path / "kv")
    m2 = g.MapReduce(device=dev)
    assert m2.load(tmp_path / "kv") == 800
    assert m2.kv.kdata.device.type == torch.device(dev).type
    assert m2.kv_pairs() == mr.kv_pairs()
    mr.collate()
    mr.save(tmp_path / "kmv")
    m3 = g.MapReduce(device=dev)
    assert m3.load(tmp_path / "kmv") == 17
    assert m3.kmv_pairs() == mr.kmv_pairs()
    # a restarted pipeline continues from the checkpoint
    assert m3.reduce("count") == 17
    assert sum(int.from_bytes(v, "little") for _, v in m3.kv_pairs()) == 800


@pytest.mark.parametrize("dev", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_spill_unspill_roundtrip(dev):
    mr = g.MapReduce(device=dev)
    _fill(mr)
    before = mr.kv_pairs()
    mr.spill()
    assert mr.kv.kdata.device.type == "cpu"
    mr.unspill()
    assert mr.kv.kdata.device.type == torch.device(dev).type
    assert mr.kv_pairs() == before
    assert mr.collate() == 17


def test_load_rejects_foreign_file(tmp_path):
    p = tmp_path / "junk"
    p.write_bytes(b"not a checkpoint")
    with pytest.raises(RuntimeError):
        g.MapReduce().load(p)


def test_verbosity_and_timer_output(capsys):
    mr = g.MapReduce()
    mr.verbosity = 1
    mr.timer = 1
    _fill(mr)
    mr.collate()
    mr.cummulative_stats(1, 0)
    out = capsys.readouterr().out
    assert "Map time (secs) =" in out
    assert "Map KV = 800 pairs" in out
    assert "Collate KMV = 17 pairs" in out
    assert "Cummulative hi-water mem" in out


@pytest.mark.parametrize("dev", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_outofcore_disk_tier(tmp_path, dev):
    """outofcore=1 (the reference's forced out-of-core mode): every op's result
    goes to fpath/mrmpi.<kv|kmv>.* and is read back by the next op; results
    equal the in-memory run and the files are gone afterwards"""
    import os

    def pipeline(mr, other):
        _fill(mr)
        mr.collate()
        mr.reduce("count")
        mr.sort_values(-1)
        other.map_mr(mr, lambda i, k, v, kv: kv.add(k, v))   # reads an MR that sits on disk
        return other.kv_pairs()

    ref = pipeline(g.MapReduce(device=dev), g.MapReduce(device=dev))
    mr, other = g.MapReduce(device=dev), g.MapReduce(device=dev)
    for m in (mr, other):
        m.outofcore = 1
        m.fpath = str(tmp_path)
    _fill(mr)
    assert mr.on_disk and any(f.startswith("mrmpi.kv.") for f in os.listdir(tmp_path))
    mr.collate()
    assert mr.on_disk and any(f.startswith("mrmpi.kmv.") for f in os.listdir(tmp_path))
    mr.reduce("count")
    mr.sort_values(-1)
    other.map_mr(mr, lambda i, k, v, kv: kv.add(k, v))
    assert other.kv_pairs() == ref
    del mr, other
    import gc
    gc.collect()
    assert [f for f in os.listdir(tmp_path) if f.startswith("mrmpi.")] == []


def test_spill_disk_manual(tmp_path):
    mr = g.MapReduce(device="cpu")
    mr.fpath = str(tmp_path)
    _fill(mr)
    before = mr.kv_pairs()
    mr.spill_disk()
    assert mr.on_disk
    assert mr.kv_pairs() == before and not mr.on_disk     # reading brings it back
    mr.spill_disk()
    assert mr.collate() == 17 and not mr.on_disk
