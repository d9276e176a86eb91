"""cubed_amd -- an MI355X-native execution path for Cubed's blockwise /
reduction / rechunk primitives, behind the reference's own API
(``cubed.core.ops``, ``Spec``, ``Plan.execute(executor=...)``).

Plans are built in Python exactly as in rsignell/cubed; the
``GpuDagExecutor`` lowers each fused pipeline to one launch of a
hand-written HIP kernel (libcubed_amd.so, C ABI in include/cubed_amd.h) on
HBM-resident chunk slabs.  See DESIGN.md.
"""

__version__ = "0.1.0"

from .array_api import Array
from .core.array import compute, measure_reserved_mem, visualize
from .core.gufunc import apply_gufunc
from .core.ops import from_array, from_zarr, map_blocks, store, to_zarr
from .nan_functions import nanmean, nansum
from .runtime.types import Callback, TaskEndEvent
from .spec import Spec

__all__ = [
    "__version__", "Callback", "Array", "Spec", "TaskEndEvent", "apply_gufunc", "compute", "from_array",
    "from_zarr", "map_blocks", "measure_reserved_mem", "nanmean", "nansum", "store",
    "to_zarr", "visualize",
]
