"""GPU numerics: every HIP kernel path vs the CPU engine path (host loops with
identical semantics and output order). Run on an MI355X: pytest -m gpu."""
import numpy as np
import pytest
import torch

from gpu_mapreduce_amd import C

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _kv(keys, values, dev):
    """keys/values: list of bytes -> native KV on dev."""
    from gpu_mapreduce_amd.runtime.keyvalue import KeyValue
    kv = KeyValue(dev)
    for k, v in zip(keys, values):
        kv.add(k, v)
    return kv.finish()


def _col(data, off, w, n):
    d = bytes(data.cpu().numpy())
    if w >= 0:
        return [d[i * w:(i + 1) * w] for i in range(n)]
    o = off.cpu().tolist()
    return [d[o[i]:o[i + 1]] for i in range(n)]


def _kv_rows(kv):
    return list(zip(_col(kv.kdata, kv.koff, kv.kw, kv.n), _col(kv.vdata, kv.voff, kv.vw, kv.n)))


def _kmv_rows(kmv):
    keys = _col(kmv.keys.kdata, kmv.keys.koff, kmv.keys.kw, kmv.nkey)
    vals = _col(kmv.vdata, kmv.voff, kmv.vw, kmv.nval)
    seg = kmv.seg.cpu().tolist()
    return [(keys[i], vals[seg[i]:seg[i + 1]]) for i in range(kmv.nkey)]


def test_native_lib_is_hip():
    import gpu_mapreduce_amd as g
    assert torch.cuda.is_available()
    assert g.so_path().endswith(".so")
    assert C.hip_compiled()


@pytest.mark.parametrize("n", [0, 1, 2047, 2048, 2049, 300_000, 5_000_001])
def test_scan(n):
    x = torch.randint(0, 1000, (n,), dtype=torch.int32)
    got = C.exclusive_scan(x.to(DEV)).cpu()
    ref = C.exclusive_scan(x)
    assert torch.equal(got, ref)
    x64 = x.long() * 1_000_003
    assert torch.equal(C.exclusive_scan(x64.to(DEV)).cpu(), C.exclusive_scan(x64))


@pytest.mark.parametrize("n,bits", [(1, 64), (1000, 16), (70_000, 32), (1_000_003, 64), (3_000_000, 26)])
def test_radix_sort_stable(n, bits):
    g = torch.Generator().manual_seed(n)
    k = torch.randint(0, 2 ** 62, (n,), generator=g, dtype=torch.int64)
    if bits < 64:
        k = k & ((1 << bits) - 1)
    k[: n // 3] = k[0]  # many duplicates -> stability matters
    v = torch.arange(n, dtype=torch.int32)
    kg, vg, _ = C.radix_sort_pairs(k.to(DEV), v.to(DEV), 0, 64)
    kc, vc, _ = C.radix_sort_pairs(k, v, 0, 64)
    assert torch.equal(kg.cpu(), kc)
    assert torch.equal(vg.cpu(), vc)


@pytest.mark.parametrize("n,bits,skip", [(2047, 64, False), (2049, 20, False), (5_000_000, 64, False),
                                         (40_000_000, 40, True), (40_000_000, 64, False)])
def test_radix_onesweep_large_vs_torch(n, bits, skip):
    """one-sweep passes (decoupled look-back across ~20 K tiles) at bench
    sizes, with and without the host-side trivial-pass skip; oracle: torch's
    stable sort of the same keys on the device"""
    g = torch.Generator(device=DEV).manual_seed(n + bits)
    k = torch.randint(0, 2 ** 62, (n,), generator=g, dtype=torch.int64, device=DEV)
    if bits < 64:
        k &= (1 << bits) - 1
    k[: n // 5] = k[n // 2]
    v = torch.arange(n, dtype=torch.int32, device=DEV)
    kg, vg, passes = C.radix_sort_pairs(k, v, 0, bits, skip)
    ks, order = torch.sort(k, stable=True)
    assert torch.equal(kg, ks)
    assert torch.equal(vg.long(), order)
    assert passes == (bits + 7) // 8


def test_hashlittle_device_matches_host():
    keys = [b"", b"a", b"Four score and seven years ago", bytes(range(200))] + \
           [np.random.default_rng(1).bytes(i) for i in range(1, 40)]
    kv_h = _kv(keys, [b""] * len(keys), "cpu")
    kv_d = kv_h.to(DEV)
    for seed in (0, 1, 8):
        assert torch.equal(C.hash32_keys(kv_d, seed).cpu(), C.hash32_keys(kv_h, seed))
    assert torch.equal(C.hash64_keys(kv_d).cpu(), C.hash64_keys(kv_h))
    # fixed width
    t = torch.randint(0, 255, (5000, 12), dtype=torch.uint8)
    f = C.make_kv(t, None, torch.empty(0, dtype=torch.uint8), None, 5000, "cpu")
    assert torch.equal(C.hash32_keys(f.to(DEV), 3).cpu(), C.hash32_keys(f, 3))
    assert torch.equal(C.hash64_keys(f.to(DEV)).cpu(), C.hash64_keys(f))


def _rand_words(n, vocab, seed):
    rng = np.random.default_rng(seed)
    words = [(b"w%d" % i) * (1 + i % 7) + b"\0" for i in range(vocab)]
    ids = rng.zipf(1.3, n) % vocab
    return [words[i] for i in ids]


@pytest.mark.parametrize("kind", ["u64", "edge", "var"])
def test_convert_matches_cpu(kind):
    rng = np.random.default_rng(0)
    n = 200_000
    if kind == "u64":
        k = torch.from_numpy(rng.integers(0, 5000, n).astype(np.int64))
        kv = C.make_kv(k, None, torch.arange(n, dtype=torch.int32), None, n, "cpu")
    elif kind == "edge":
        k = torch.from_numpy(rng.integers(0, 300, (n, 2)).astype(np.int64))
        kv = C.make_kv(k, None, torch.arange(n, dtype=torch.float64), None, n, "cpu")
    else:
        keys = _rand_words(n, 3000, 1)
        kv = _kv(keys, [b"v%d" % (i % 13) for i in range(n)], "cpu")
    kc, sc = C.convert(kv)
    kg, sg = C.convert(kv.to(DEV))
    assert sc.collisions == 0 and sg.collisions == 0
    assert _kmv_rows(kg) == _kmv_rows(kc)


def test_convert_hash_collision_fallback():
    keys = _rand_words(20_000, 500, 2)
    kv = _kv(keys, [b""] * len(keys), "cpu")
    kg, sg = C.convert(kv.to(DEV), 4)   # only 16 hash buckets -> forced collisions
    assert sg.collisions > 0
    rows = _kmv_rows(kg)
    assert len(rows) == len(set(keys))
    from collections import Counter
    cnt = Counter(keys)
    assert all(len(v) == cnt[k] for k, v in rows)


@pytest.mark.parametrize("dtype,np_t", [("int32", np.int32), ("int64", np.int64), ("float32", np.float32),
                                        ("float64", np.float64)])
@pytest.mark.parametrize("op", ["sum", "min", "max"])
def test_reduce_builtin(dtype, np_t, op):
    rng = np.random.default_rng(3)
    n = 100_000
    k = np.concatenate([rng.integers(0, 2000, n - 5000), np.full(5000, 7)]).astype(np.int64)  # one long segment
    v = (rng.standard_normal(n) * 100).astype(np_t)
    kv = C.make_kv(torch.from_numpy(k), None, torch.from_numpy(v), None, n, "cpu")
    kc, _ = C.convert(kv)
    kg, _ = C.convert(kv.to(DEV))
    rc = C.reduce_builtin(kc, op, dtype)
    rg = C.reduce_builtin(kg, op, dtype)
    a = np.frombuffer(bytes(rc.vdata.numpy()), dtype=np_t)
    b = np.frombuffer(bytes(rg.vdata.cpu().numpy()), dtype=np_t)
    if op == "sum" and dtype.startswith("float"):
        np.testing.assert_allclose(b, a, rtol=1e-4, atol=1e-2)
    else:
        assert np.array_equal(a, b)
    for o in ("count", "first", "last"):
        assert _kv_rows(C.reduce_builtin(kg, o, "")) == _kv_rows(C.reduce_builtin(kc, o, ""))


@pytest.mark.parametrize("flag", [1, -1, 2, -2, 3, -3, 4, -4, 5, -5, 6])
def test_sort_flags(flag):
    rng = np.random.default_rng(abs(flag))
    n = 50_000
    if abs(flag) in (1, 3):
        raw = rng.standard_normal(n).astype(np.float32 if abs(flag) == 3 else np.float64)
        v = (raw * 1000).astype(np.int32) if abs(flag) == 1 else raw
        col = torch.from_numpy(np.ascontiguousarray(v))
    elif abs(flag) in (2, 4):
        v = rng.integers(0, 2 ** 63, n).astype(np.uint64) if abs(flag) == 2 else rng.standard_normal(n)
        col = torch.from_numpy(v.view(np.int64) if abs(flag) == 2 else v)
    else:
        words = [b"prefix_shared_%d\0" % i for i in rng.integers(0, 10 ** 6, n)]
        kv = _kv(words, [b"x"] * n, "cpu")
        a = _kv_rows(C.sort_kv(kv, flag, False))
        b = _kv_rows(C.sort_kv(kv.to(DEV), flag, False))
        assert a == b
        keys = [r[0] for r in b]
        assert keys == sorted(words, reverse=flag < 0)
        return
    kv = C.make_kv(col, None, torch.arange(n, dtype=torch.int32), None, n, "cpu")
    a = _kv_rows(C.sort_kv(kv, flag, False))
    b = _kv_rows(C.sort_kv(kv.to(DEV), flag, False))
    assert a == b


def test_map_urls_and_words_match_cpu():
    from gpu_mapreduce_amd.utils import synth
    t = synth.html_file(3_000_000, seed=4, nurl=5000, device="cpu")
    buf = synth.pad_text(t)
    a = _kv_rows(C.map_urls(buf, t.numel(), 3))
    b = _kv_rows(C.map_urls(buf.to(DEV), t.numel(), 3))
    assert len(a) > 1000 and a == b
    w = synth.pad_text(synth.zipf_text(2_000_000, seed=2))
    a = _kv_rows(C.map_words(w, w.numel() - 64))
    b = _kv_rows(C.map_words(w.to(DEV), w.numel() - 64))
    assert len(a) > 1000 and a == b


def test_map_words_separators_and_tile_edges():
    """one-pass word keys (text.hip k_tok_emit2): runs of mixed separators,
    leading / trailing separators, words across 16-byte thread and 4 KiB tile
    boundaries, a 10 KB word, a word ending exactly at n (bytes past n are
    separators even when the padding is not)"""
    import random
    from gpu_mapreduce_amd.utils import synth
    rng = random.Random(7)
    parts = [b"  \t"]
    for i in range(40000):
        parts.append(b"w%d" % rng.randrange(5000) + b"x" * rng.choice([0, 0, 1, 5, 13, 30]))
        parts.append(rng.choice([b" ", b" ", b"\n", b"\t\r ", b"   \f  "]))
    parts.append(b"L" * 10000)
    parts.append(b" tail")
    raw = b"".join(parts)
    t = torch.frombuffer(bytearray(raw), dtype=torch.uint8)
    for cut in (len(raw), len(raw) - 2, 4096 * 7 + 3):
        w = synth.pad_text(t[:cut].clone())
        w[cut:cut + 8] = ord("z")  # non-separators right past n must not extend the last word
        a = _kv_rows(C.map_words(w, cut))
        b = _kv_rows(C.map_words(w.to(DEV), cut))
        assert len(a) > 100 and a == b, cut


def test_rmat_bit_exact():
    a = C.map_rmat(100_000, 16, 0.57, 0.19, 0.19, 0.05, 0.0, 12345, 777, "cpu")
    b = C.map_rmat(100_000, 16, 0.57, 0.19, 0.19, 0.05, 0.0, 12345, 777, DEV)
    assert torch.equal(a.kdata, b.kdata.cpu())
    e = a.kdata.view(torch.int64).view(-1, 2)
    assert int(e.max()) < 2 ** 16


@pytest.mark.parametrize("streams", [0, 1, 3])
def test_inverted_index_end_to_end_gpu(streams):
    """the staging ring depth (MapReduce.streams: 0 auto, 1 serial, 3) never
    changes the output bytes"""
    import gpu_mapreduce_amd as g
    from gpu_mapreduce_amd.models.inverted_index import InvertedIndex, reference_inverted_index
    from gpu_mapreduce_amd.utils import synth
    files = synth.html_corpus(4_000_000, file_bytes=1_000_000, seed=9, nurl=20_000)
    mr = g.MapReduce(g.Comm(device="cuda"))
    mr.streams = streams
    app = InvertedIndex(mr, [(n, t.pin_memory()) for n, t in files])
    app.run()
    assert app.nbuf == (streams or 3)
    got = {}
    for line in app.output_lines():
        url, rest = line.split("\t")
        got[url.encode()] = sorted(rest.split())
    assert got == reference_inverted_index(files)


def test_gather_var_and_expand():
    keys = _rand_words(50_000, 1000, 5)
    kv = _kv(keys, [b"val%d" % i for i in range(len(keys))], "cpu")
    perm = torch.randperm(len(keys)).to(torch.int32)
    assert _kv_rows(C.gather(kv.to(DEV), perm.to(DEV))) == _kv_rows(C.gather(kv, perm))
    kc, _ = C.convert(kv)
    kg, _ = C.convert(kv.to(DEV))
    assert _kv_rows(C.expand(kg)) == _kv_rows(C.expand(kc))


def test_inverted_index_bench_scale_gpu():
    """bench shape (128 MiB part files, the bench's URL density), 512 MiB:
    the pipelined + grouped InvertedIndex output equals the Python oracle,
    and a second job on the same files gives the same bytes (deterministic
    order of keys and of each key's files)"""
    import gpu_mapreduce_amd as g
    from gpu_mapreduce_amd.models.inverted_index import InvertedIndex, reference_inverted_index
    from gpu_mapreduce_amd.utils import synth
    files = synth.html_corpus(512 << 20, file_bytes=128 << 20, seed=1, device=DEV, link_gap=200)
    files = [(n, t.cpu().pin_memory()) for n, t in files]
    comm = g.Comm(device="cuda")
    outs = []
    # jobs 0 and 1 prefetch the next job's first file (a job pipeline), job 2
    # finds its first file already staged, job 3 runs alone
    for j in range(4):
        mr = g.MapReduce(comm)
        app = InvertedIndex(mr, files, prefetch_next=files if j < 2 else None)
        app.run()
        assert mr.last_convert.grouped == 1
        app.output_ready()
        outs.append(bytes(app.output.numpy()))
    assert outs[0] == outs[1] == outs[2] == outs[3]
    got = {}
    for line in outs[0].decode("utf-8", "replace").splitlines():
        url, rest = line.split("\t")
        got[url.encode()] = sorted(rest.split())
    assert got == reference_inverted_index(files)


@pytest.mark.parametrize("dtype,np_t", [("int64", np.int64), ("float64", np.float64)])
@pytest.mark.parametrize("op", ["sum", "max"])
def test_reduce_builtin_hub_two_level_carry(dtype, np_t, op):
    """12 M values, one key holding 8 M of them: the segmented reduce spans
    2900 tiles, whose carries are folded in two levels (k_carry_fold)"""
    rng = np.random.default_rng(5)
    n, hub = 12_000_000, 8_000_000
    k = np.concatenate([rng.integers(0, 500_000, n - hub), np.full(hub, 123_456)]).astype(np.int64)
    v = rng.integers(-1000, 1000, n).astype(np_t)
    kv = C.make_kv(torch.from_numpy(k), None, torch.from_numpy(v), None, n, DEV)
    kg, _ = C.convert(kv)
    rg = C.reduce_builtin(kg, op, dtype)
    keys = np.frombuffer(bytes(rg.kdata.cpu().numpy()), dtype=np.int64)
    got = np.frombuffer(bytes(rg.vdata.cpu().numpy()), dtype=np_t)
    order = np.argsort(k, kind="stable")
    ks, vs = k[order], v[order]
    heads = np.concatenate([[0], np.nonzero(np.diff(ks))[0] + 1])
    ref = (np.add if op == "sum" else np.maximum).reduceat(vs, heads)
    ref_keys = ks[heads]
    pos = np.argsort(keys)
    assert np.array_equal(keys[pos], ref_keys)
    assert np.array_equal(got[pos], ref)  # integer-valued: exact in float64 too
