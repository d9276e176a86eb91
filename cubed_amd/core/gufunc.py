"""apply_gufunc (cubed/core/gufunc.py:7-148, itself cut down from dask's):
validate a generalized-ufunc signature against the chunked inputs and apply
``func`` with ``blockwise`` over all output dims.  ``func`` lowers like any
other blockwise function (numpy ufuncs and cubed_amd chunk programs run on
the MI355X executor; anything else is refused at execute time)."""

import re

import numpy as np

_DIMNAME = r"\w+"
_CORE_DIMS = r"(?:{0}(?:,{0})*)?".format(_DIMNAME)
_ARG = r"\({}\)".format(_CORE_DIMS)
_ARGS = r"(?:{0}(?:,{0})*)?".format(_ARG)
_SIGNATURE = r"^{0}->{0}$".format(_ARGS)


def parse_gufunc_signature(signature):
    """``"(i,j),(j)->(i)"`` -> ([("i", "j"), ("j",)], ("i",)); several
    outputs give a list of tuples (numpy's gufunc signature grammar)."""
    signature = re.sub(r"\s+", "", signature)
    if not re.match(_SIGNATURE, signature):
        raise ValueError(f"Not a valid gufunc signature: {signature}")
    ins, outs = signature.split("->")
    in_dims = [tuple(re.findall(_DIMNAME, a)) for a in re.findall(_ARG, ins)]
    out_dims = [tuple(re.findall(_DIMNAME, a)) for a in re.findall(_ARG, outs)]
    return in_dims, (out_dims[0] if len(out_dims) == 1 else out_dims)


def apply_gufunc(func, signature, *args, axes=None, axis=None, output_dtypes=None,
                 output_sizes=None, vectorize=None, **kwargs):
    from .ops import blockwise

    if not isinstance(signature, str):
        raise TypeError("`signature` has to be of type string")
    in_core, out_core = parse_gufunc_signature(signature)
    if isinstance(out_core, list):
        raise NotImplementedError(
            "Multiple outputs are not yet supported, see https://github.com/tomwhite/cubed/issues/69")
    if vectorize:
        func = np.vectorize(func, signature=signature, otypes=output_dtypes)
    output_sizes = dict(output_sizes or {})
    if len(in_core) != len(args):
        raise ValueError(
            f"According to `signature`, `func` requires {len(in_core)} arguments, but {len(args)} given")

    nloop = [len(a.shape) - len(cd) for a, cd in zip(args, in_core)]
    maxloop = max(nloop) if nloop else 0
    core_shapes = {}
    for a, n, cd in zip(args, nloop, in_core):
        core_shapes.update(zip(cd, a.shape[n:]))
    core_shapes.update(output_sizes)
    loop_dims = [tuple(f"__loopdim{d}__" for d in range(maxloop - n, maxloop)) for n in nloop]
    in_dims = [lp + cd for lp, cd in zip(loop_dims, in_core)]
    out_loop = max(loop_dims, key=len) if loop_dims else ()

    sizes, chunksizes = {}, {}
    for dims, a in zip(in_dims, args):
        for dim, size, cs in zip(dims, a.shape, a.chunks):
            sizes.setdefault(dim, []).append(size)
            chunksizes.setdefault(dim, []).append(cs)
    for dim, ss in sizes.items():
        if set(ss) | {1} != {1, max(ss)}:
            raise ValueError(f"Dimension `'{dim}'` with different lengths in arrays")
        cs = chunksizes[dim]
        if dim in core_shapes and cs[0][0] < core_shapes[dim]:
            raise ValueError(
                f"Core dimension `'{dim}'` consists of multiple chunks. To fix, rechunk into a single "
                "chunk along this dimension or set `allow_rechunk=True`, but beware that this may "
                "increase memory usage significantly.")
        relevant = {c for s, c in zip(ss, cs) if s > 1}
        if len(relevant) > 1:
            raise ValueError(f"Dimension `'{dim}'` with different chunksize present")

    arginds = [x for a, d in zip(args, in_dims) for x in (a, d)]
    out_ind = out_loop + out_core
    return blockwise(func, out_ind, *arginds, dtype=output_dtypes, new_axes=output_sizes, **kwargs)
