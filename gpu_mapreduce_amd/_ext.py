"""Loader for the native engine extension (gpu_mapreduce_amd/_C*.so).

There is deliberately NO pure-Python fallback: every data-plane op runs in
the native engine (HIP/CDNA4 kernels on MI355X, host loops on CPU). If the
extension is missing the import fails loudly with the build command.
"""
import importlib
import os

_here = os.path.dirname(os.path.abspath(__file__))


def _load():
    try:
        import torch  # noqa: F401  (loads libtorch / HIP runtime first)
        return importlib.import_module("gpu_mapreduce_amd._C")
    except ImportError as e:  # pragma: no cover - exercised only on broken installs
        raise ImportError(
            "gpu_mapreduce_amd native extension not built. Run:\n"
            "  PYTORCH_ROCM_ARCH=gfx950 python setup.py build_ext --inplace\n"
            f"(from {os.path.dirname(_here)}); original error: {e}"
        ) from e


C = _load()

# Device allocator of the process, chosen before anything allocates device
# memory:
#  * MRH_GUARD=1: the guarded (canaried) allocator (csrc/engine/guardalloc.h);
#  * default: the engine's HBM page pool (csrc/engine/hbmpool.h) — per-stream
#    size-class caches over stream-ordered HIP memory pools, with the hard cap
#    MapReduce ops with a page budget (maxpage x memsize / hbm_budget) run
#    under. It needs this package imported before the first device allocation
#    of the process; otherwise the ATen caching allocator stays (a requested
#    MRH_HBM_POOL=1 then fails loudly). MRH_HBM_POOL=0 keeps the ATen
#    caching allocator.
_POOL = os.environ.get("MRH_HBM_POOL", "")
if os.environ.get("MRH_GUARD", "0") not in ("", "0"):
    C.install_alloc_guard()
elif _POOL != "0":
    import torch as _torch
    # device_count() does not initialise the device allocator (is_available()-style probes may)
    if _torch.cuda.device_count() > 0 and not C.hbm_pool_install() and _POOL == "1":
        raise RuntimeError("MRH_HBM_POOL=1: device memory was allocated before gpu_mapreduce_amd was imported; "
                           "import it first so the page pool can become the device allocator")


def so_path():
    """Path of the loaded native library (used by tests / smoke to prove the
    HIP path is the one that ran)."""
    return C.__file__
