"""apply_gufunc (cubed/core/gufunc.py): signature parsing and the
validation errors of the reference (tests/test_gufunc.py), on CPU; the
GPU cases run the reference's elementwise gufuncs through tracing."""

import numpy as np
import pytest

import cubed_amd as cubed
from cubed_amd import apply_gufunc
from cubed_amd.core.gufunc import parse_gufunc_signature


def test_parse_signature():
    assert parse_gufunc_signature("(i,j),(j)->(i)") == ([("i", "j"), ("j",)], ("i",))
    assert parse_gufunc_signature("(),()->()") == ([(), ()], ())
    assert parse_gufunc_signature("(i)->(),()") == ([("i",)], [(), ()])
    with pytest.raises(ValueError, match="Not a valid gufunc signature"):
        parse_gufunc_signature("(i,j)->(i")


def test_validation_errors():
    spec = cubed.Spec(allowed_mem="1GB")
    a = cubed.from_array(np.arange(6).reshape(2, 3), chunks=(1, 2), spec=spec)
    with pytest.raises(TypeError):
        apply_gufunc(np.add, 3, a, a)
    with pytest.raises(ValueError, match="requires 2 arguments"):
        apply_gufunc(np.add, "(),()->()", a)
    with pytest.raises(ValueError, match="consists of multiple chunks"):
        apply_gufunc(np.sum, "(i)->()", a, output_dtypes=a.dtype)
    with pytest.raises(NotImplementedError, match="Multiple outputs"):
        apply_gufunc(np.divmod, "(),()->(),()", a, a)
    b = cubed.from_array(np.arange(6).reshape(2, 3), chunks=(2, 1), spec=spec)
    with pytest.raises(ValueError, match="different chunksize"):
        apply_gufunc(np.add, "(),()->()", a, b, output_dtypes=a.dtype)
    c = cubed.from_array(np.arange(4).reshape(2, 2), chunks=(1, 2), spec=spec)
    with pytest.raises(ValueError, match="different lengths"):
        apply_gufunc(np.add, "(),()->()", a, c, output_dtypes=a.dtype)


@pytest.mark.gpu
def test_apply_gufunc_reference_elementwise(gpu_executor):
    spec = cubed.Spec(allowed_mem="1GB", executor=gpu_executor)

    def add(x, y):
        return x + y

    a = cubed.from_array(np.array([1, 2, 3]), chunks=2, spec=spec)
    b = cubed.from_array(np.array([1, 2, 3]), chunks=2, spec=spec)
    assert np.array_equal(apply_gufunc(add, "(),()->()", a, b, output_dtypes=a.dtype).compute(), [2, 4, 6])
    z = apply_gufunc(lambda x: 2 * x, "()->()", a, output_dtypes=int)
    assert z.chunks == ((2, 1),)
    assert np.array_equal(z.compute(), [2, 4, 6])
    c = cubed.from_array(np.array([1, 2, 3]), chunks=3, spec=spec)
    z = apply_gufunc(lambda x: 2 * x, "(i)->(i)", c, output_dtypes=int)
    assert z.chunks == ((3,),)
    assert np.array_equal(z.compute(), [2, 4, 6])
