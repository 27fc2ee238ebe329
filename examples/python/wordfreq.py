"""Word frequency with the reference-style `mrmpi` Python interface
(the job of the reference's examples/wordfreq.py, Python 3, on the native
engine). Run: python examples/python/wordfreq.py file1 dir2 ...
Multi-GPU: torchrun --nproc-per-node N --master-addr 127.0.0.1 examples/python/wordfreq.py ..."""
import sys
import time

from gpu_mapreduce_amd.mrmpi import mrmpi
from gpu_mapreduce_amd.parallel.comm import init


def main(files, ntop=10):
    comm = init()

    def fileread(itask, name, mr):
        with open(name, errors="replace") as f:
            for word in f.read().split():
                mr.add(word, None)

    def total(key, mvalue, mr):
        mr.add(key, len(mvalue))

    def ncompare(a, b):
        return (a < b) - (a > b)          # descending counts

    state = {"n": 0}

    def keep(itask, key, value, mr):
        state["n"] += 1
        if state["n"] <= ntop:
            mr.add(key, value)

    mr = mrmpi(comm)
    t0 = time.perf_counter()
    nwords = mr.map_file(files, 0, 1, 0, fileread)
    mr.collate()
    nunique = mr.reduce(total)
    mr.sort_values(ncompare)
    top = mrmpi(comm)
    top.map_mr(mr, keep)
    top.gather(1)
    top.sort_values(ncompare)
    dt = time.perf_counter() - t0
    result = top.pairs()[:ntop]
    if comm.rank == 0:
        for word, count in result:
            print(count, word)
        print(f"{nwords} total words, {nunique} unique words")
        print(f"Time to process {len(files)} inputs = {dt:.3f} (secs)")
    return nwords, nunique, result


if __name__ == "__main__":
    main(sys.argv[1:])
