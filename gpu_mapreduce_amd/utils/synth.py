"""Synthetic inputs with the shapes of the reference workloads (no datasets are
available offline):

* `html_corpus`: Wikipedia-like HTML "part" files for InvertedIndex
  (reference cuda/InvertedIndex.cu:284-304 reads 128 MB `part-%05d` files and
  extracts `<a href="...">` URLs). Links are drawn from a Zipf-distributed
  URL vocabulary, separated by filler text/markup; the mean link gap is a
  parameter (default 200 B, about the link density of Wikipedia HTML).
* `zipf_text`: whitespace-separated words with a Zipf frequency law for
  wordfreq (the reference's examples/words/text.txt is missing).

Generation is vectorised with torch and can run on the GPU (fast) or CPU;
every byte is a pure function of (seed, rank) so runs are reproducible.
"""
from __future__ import annotations

import math

import torch

_LETTERS = torch.frombuffer(bytearray(b"abcdefghijklmnopqrstuvwxyz"), dtype=torch.uint8)
_URL_CHARS = torch.frombuffer(bytearray(b"abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789_"),
                              dtype=torch.uint8)
_FILLER_WORDS = [b"the", b"of", b"and", b"in", b"was", b"<p>", b"</p>", b"<b>", b"</b>", b"is", b"for",
                 b"<span class=\"x\">", b"</span>", b"on", b"with", b"as", b"by", b"<li>", b"</li>",
                 b"history", b"city", b"river", b"population", b"century", b"<br/>", b"\n"]


def _zipf_ids(n, vocab, s, gen, device):
    """n samples of a truncated Zipf(s) over [0, vocab) by inverse CDF."""
    ranks = torch.arange(1, vocab + 1, dtype=torch.float64, device=device)
    w = ranks.pow(-s)
    cdf = torch.cumsum(w, 0)
    cdf /= cdf[-1].clone()
    u = torch.rand(n, generator=gen, dtype=torch.float64, device=device)
    return torch.searchsorted(cdf, u).clamp_(max=vocab - 1)


def _gen(seed, device):
    g = torch.Generator(device=device)
    g.manual_seed(int(seed))
    return g


def _assemble(pool: torch.Tensor, src_off: torch.Tensor, lens: torch.Tensor) -> torch.Tensor:
    """Concatenate pieces pool[src_off[i] : src_off[i]+lens[i]] (vectorised)."""
    total = int(lens.sum().item())
    starts = torch.cumsum(lens, 0) - lens
    piece = torch.repeat_interleave(torch.arange(lens.numel(), device=pool.device), lens, output_size=total)
    within = torch.arange(total, device=pool.device) - starts[piece]
    return pool[src_off[piece] + within]


def url_vocab(nurl, seed=7, device="cpu", min_len=8, max_len=60):
    g = _gen(seed, device)
    lens = torch.randint(min_len, max_len + 1, (nurl,), generator=g, device=device)
    chars = _URL_CHARS.to(device)[torch.randint(0, len(_URL_CHARS), (int(lens.sum()),), generator=g, device=device)]
    prefix = b"http://en.wikipedia.org/wiki/"
    return chars, lens, prefix


def html_file(nbytes, seed, device="cpu", nurl=1 << 20, link_gap=200, zipf_s=1.0, vocab=None):
    """One synthetic HTML file of ~nbytes bytes (uint8 tensor, exact length nbytes)."""
    g = _gen(seed, device)
    chars, ulens, prefix = vocab if vocab is not None else url_vocab(nurl, device=device)
    nurl = ulens.numel()
    uoff = torch.cumsum(ulens, 0) - ulens
    filler_words = torch.cat([torch.frombuffer(bytearray(w + b" "), dtype=torch.uint8) for w in _FILLER_WORDS])
    # random filler pool built from words (no '<a href="' inside it)
    nfw = 1 << 16
    widx = torch.randint(0, len(_FILLER_WORDS), (nfw,), generator=_gen(seed + 1, "cpu"))
    fpool = torch.cat([torch.frombuffer(bytearray(_FILLER_WORDS[i] + b" "), dtype=torch.uint8) for i in widx.tolist()])
    fpool = fpool.to(device)
    fpl = fpool.numel()
    mean_unit = link_gap
    nlinks = max(1, int(nbytes / mean_unit))
    uid = _zipf_ids(nlinks, nurl, zipf_s, g, device)
    # per link: filler gap, anchor text
    gap = torch.randint(mean_unit // 4, max(mean_unit // 4 + 1, mean_unit * 3 // 4), (nlinks,), generator=g,
                        device=device)
    anch = torch.randint(3, 20, (nlinks,), generator=g, device=device)
    fo = torch.randint(0, fpl - 64 - mean_unit, (nlinks,), generator=g, device=device)
    ao = torch.randint(0, fpl - 64, (nlinks,), generator=g, device=device)
    # combined pool: [filler | constant strings | url chars]
    consts = torch.frombuffer(bytearray(b'<a href="' + prefix + b'">' + b"</a>"), dtype=torch.uint8).to(device)
    c0 = fpl
    pool = torch.cat([fpool, consts, chars])
    p_open, l_open = c0, 9 + len(prefix)
    p_close, l_close = c0 + l_open, 2
    p_end, l_end = c0 + l_open + 2, 4
    ubase = c0 + consts.numel()
    src = torch.stack([fo, torch.full_like(fo, p_open), ubase + uoff[uid], torch.full_like(fo, p_close), ao,
                       torch.full_like(fo, p_end)], 1).reshape(-1)
    lens = torch.stack([gap, torch.full_like(gap, l_open), ulens[uid], torch.full_like(gap, l_close), anch,
                        torch.full_like(gap, l_end)], 1).reshape(-1)
    text = _assemble(pool, src, lens)
    if text.numel() >= nbytes:
        return text[:nbytes].contiguous()
    pad = fpool[: nbytes - text.numel()] if nbytes - text.numel() <= fpl else \
        fpool.repeat(math.ceil((nbytes - text.numel()) / fpl))[: nbytes - text.numel()]
    return torch.cat([text, pad])


def html_corpus(total_bytes, file_bytes=128 << 20, seed=0, rank=0, device="cpu", **kw):
    """List of (name, uint8 tensor) part files for one rank."""
    vocab = url_vocab(kw.pop("nurl", 1 << 20), seed=7, device=device)
    nfiles = max(1, math.ceil(total_bytes / file_bytes))
    out = []
    left = total_bytes
    for f in range(nfiles):
        nb = min(file_bytes, left)
        left -= nb
        fid = rank * nfiles + f
        out.append((f"part-{fid:05d}", html_file(nb, seed * 1000003 + fid, device=device, vocab=vocab, **kw)))
    return out


def zipf_text(nbytes, seed=0, device="cpu", vocab=1 << 16, s=1.1, min_len=1, max_len=12):
    """~nbytes of whitespace-separated Zipf-distributed lowercase words."""
    g = _gen(seed, device)
    wl = torch.randint(min_len, max_len + 1, (vocab,), generator=_gen(1234, device), device=device)
    chars = _LETTERS.to(device)[torch.randint(0, 26, (int(wl.sum()),), generator=_gen(4321, device), device=device)]
    sep = torch.tensor([32, 10], dtype=torch.uint8, device=device)
    pool = torch.cat([chars, sep])
    woff = torch.cumsum(wl, 0) - wl
    mean = float(wl.float().mean()) + 1
    n = max(1, int(nbytes / mean))
    ids = _zipf_ids(n, vocab, s, g, device)
    nl = (torch.rand(n, generator=g, device=device) < 0.05).long()
    src = torch.stack([woff[ids], chars.numel() + nl], 1).reshape(-1)
    lens = torch.stack([wl[ids], torch.ones_like(ids)], 1).reshape(-1)
    text = _assemble(pool, src, lens)
    return text[:nbytes].contiguous() if text.numel() >= nbytes else torch.cat(
        [text, torch.full((nbytes - text.numel(),), 32, dtype=torch.uint8, device=device)])


def pad_text(t: torch.Tensor, pad=64) -> torch.Tensor:
    """Copy a text tensor into a buffer with `pad` trailing zero bytes (the
    text map kernels read 16-byte windows past the end)."""
    out = torch.zeros(t.numel() + pad, dtype=torch.uint8, device=t.device)
    out[: t.numel()] = t
    return out


def _main(argv=None):
    """Write synthetic input files for the native apps (csrc/apps):
        python -m gpu_mapreduce_amd.utils.synth html  DIR NFILES FILE_BYTES   # part-%05d HTML files
        python -m gpu_mapreduce_amd.utils.synth text  DIR NFILES FILE_BYTES   # Zipf word text files
        python -m gpu_mapreduce_amd.utils.synth ints  FILE NBYTES KEY_RANGE   # raw int32 file (IntCount)
    """
    import argparse
    import os

    ap = argparse.ArgumentParser(prog="python -m gpu_mapreduce_amd.utils.synth")
    ap.add_argument("kind", choices=["html", "text", "ints"])
    ap.add_argument("path")
    ap.add_argument("a", type=int)
    ap.add_argument("b", type=int)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--nurl", type=int, default=1 << 16)
    ap.add_argument("--device", default="cpu", help="generate on this torch device (e.g. cuda) and write from host")
    args = ap.parse_args(argv)
    dev = args.device
    if args.kind == "ints":
        g = _gen(args.seed, "cpu")
        v = torch.randint(0, args.b, (args.a // 4,), generator=g, dtype=torch.int32)
        with open(args.path, "wb") as f:
            f.write(v.numpy().tobytes())
        return
    os.makedirs(args.path, exist_ok=True)
    vocab = url_vocab(args.nurl, device=dev) if args.kind == "html" else None
    for i in range(args.a):
        if args.kind == "html":
            t = html_file(args.b, args.seed * 1000003 + i, device=dev, vocab=vocab)
            name = f"part-{i:05d}"
        else:
            t = zipf_text(args.b, seed=args.seed * 1000003 + i, device=dev)
            name = f"text-{i:05d}.txt"
        with open(os.path.join(args.path, name), "wb") as f:
            f.write(t.cpu().numpy().tobytes())


if __name__ == "__main__":
    _main()
