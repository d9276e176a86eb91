"""Array API namespace of the MI355X Cubed build (``import cubed_amd.array_api as xp``)."""

__array_api_version__ = "2022.12"

from .array_object import Array
from .constants import e, inf, nan, newaxis, pi
from .creation_functions import (
    arange,
    asarray,
    empty,
    empty_like,
    eye,
    full,
    full_like,
    linspace,
    meshgrid,
    ones,
    ones_like,
    tril,
    triu,
    zeros,
    zeros_like,
)
from .data_type_functions import astype, can_cast, finfo, iinfo, isdtype, result_type
from .dtypes import (
    bfloat16,
    bool,
    complex64,
    complex128,
    float32,
    float64,
    int8,
    int16,
    int32,
    int64,
    uint8,
    uint16,
    uint32,
    uint64,
)
from .elementwise_functions import *  # noqa: F401,F403
from .elementwise_functions import abs, round  # noqa: F401
from .linear_algebra_functions import matmul, matrix_transpose, outer, tensordot, vecdot
from .indexing_functions import take
from .manipulation_functions import (
    broadcast_arrays,
    broadcast_to,
    concat,
    expand_dims,
    flatten,
    moveaxis,
    permute_dims,
    reshape,
    squeeze,
    stack,
)
from .searching_functions import argmax, argmin, where
from .statistical_functions import max, mean, min, prod, std, sum, var
from .utility_functions import all, any
