"""Zarr source/sink I/O (reference core/ops.py:88-182, storage/zarr.py).

The ``zarr`` package is not part of this build's environment; these entry
points exist for API parity and raise a clear error until the native Zarr v2
reader/writer lands."""


def _require_zarr():
    try:
        import zarr  # noqa: F401
    except ImportError as e:
        raise ImportError(
            "Zarr I/O needs the 'zarr' package, which is not installed; use "
            "from_array / compute() to move data in and out of HBM") from e


def from_zarr(store, spec=None):
    _require_zarr()
    raise NotImplementedError("from_zarr: Zarr source reads are not lowered yet")


def to_zarr(x, store, executor=None, **kwargs):
    _require_zarr()
    raise NotImplementedError("to_zarr: Zarr sink writes are not lowered yet")


def store(sources, targets, executor=None, **kwargs):
    _require_zarr()
    raise NotImplementedError("store: Zarr sink writes are not lowered yet")
