"""Restart files in the reference's H5Part layout (libsphexa_h5part.so, sphexa_amd.h5part), CPU.

Pinned against the reference's own writer and reader: main/src/io/ifile_io_hdf5.cpp (H5PartWriter / H5PartReader)
over extern/h5part/H5Part.c, compiled serially from /root/reference into oracle/_ref/libh5part_ref.so
(oracle/Makefile, harness oracle/h5part_ref.cpp), linked to the image's serial HDF5 1.10.6:
  * a checkpoint written here (the conserved fields with the reference's names and types, the step attributes of
    ParticlesData::loadOrStoreAttributes + Box::loadOrStore) is read by the reference's H5PartReader: particle count,
    attribute names, every attribute through stepAttribute with the C++ type loadOrStoreAttributes passes (its
    readAttribute type checks apply), every field bit for bit;
  * a step written by the reference's H5PartWriter is read here bit for bit, with the reference's on-disk types;
  * several steps append to one file ("Step#0", "Step#1"), the reader's step -1 is the last.
The self round-trip test runs wherever the library is built.
"""
import ctypes as C
import os

import numpy as np
import pytest

import pyoracle as po
import sphexa_amd as sx
from sphexa_amd import h5part

REF_SO = os.path.join(os.path.dirname(po.REF_SO), "libh5part_ref.so")
ref_only = pytest.mark.skipif(not os.path.exists(REF_SO), reason="oracle/_ref/libh5part_ref.so not built")

# numpy dtype -> position in sphexa::IO::Types (ifile_io.hpp:46), the harness's type codes
IOTYPE = {np.dtype(np.float64): 0, np.dtype(np.float32): 1, np.dtype(np.int8): 2, np.dtype(np.uint8): 3,
          np.dtype(np.int32): 4, np.dtype(np.int64): 5, np.dtype(np.uint32): 6, np.dtype(np.uint64): 7}

FIELD_TYPES = {"x": np.float64, "y": np.float64, "z": np.float64, "h": np.float32, "m": np.float32,
               "temp": np.float64, "vx": np.float32, "vy": np.float32, "vz": np.float32, "x_m1": np.float32,
               "y_m1": np.float32, "z_m1": np.float32, "du_m1": np.float32, "alpha": np.float32, "id": np.uint64,
               "rung": np.uint8}


def ref_lib():
    L = C.CDLL(REF_SO)
    L.ref_h5_last_error.restype = C.c_char_p
    L.ref_h5_num_particles.restype = C.c_int64
    L.ref_h5_num_particles.argtypes = [C.c_char_p, C.c_int]
    L.ref_h5_step_attributes.argtypes = [C.c_char_p, C.c_int, C.c_char_p, C.c_int]
    L.ref_h5_read_attribute.argtypes = [C.c_char_p, C.c_int, C.c_char_p, C.c_int, C.c_void_p, C.c_int64]
    L.ref_h5_read_field.argtypes = [C.c_char_p, C.c_int, C.c_char_p, C.c_int, C.c_void_p]
    return L


def sample_state(n, seed=1):
    rng = np.random.default_rng(seed)
    out = {}
    for k, t in FIELD_TYPES.items():
        if np.dtype(t).kind == "f":
            out[k] = rng.standard_normal(n).astype(t)
        elif k == "id":
            out[k] = rng.permutation(n).astype(np.uint64) + np.uint64(1 << 40)
        else:
            out[k] = rng.integers(0, 4, n).astype(t)
    return out


def sample_attributes(it=12):
    p = sx.default_params(g=0.5)
    box = sx.make_box([-0.5, 0.5, -0.5, 0.5, -1.0, 1.0], [1, 1, 0])
    a = sx.reference_attributes(p, box, {"ttot": 0.0123, "minDt": 2.5e-4, "minDt_m1": 2.25e-4}, it, 4096)
    a["ts::numRungs"] = np.int32(3)
    a["ts::dt_m1"] = np.array([1e-4, 2e-4, 4e-4, 0.0], np.float32)
    return a


def test_self_round_trip(tmp_path):
    path = str(tmp_path / "rt.h5")
    st, at = sample_state(777), sample_attributes()
    h5part.write_step(path, st, at, mode="w")
    got, ga = h5part.read_step(path, {k: v.dtype for k, v in st.items()}, {k: np.asarray(v).dtype for k, v in at.items()})
    for k in st:
        assert np.array_equal(got[k], st[k]) and got[k].dtype == st[k].dtype, k
    for k in at:
        assert np.array_equal(np.asarray(ga[k]), np.asarray(at[k])), k
    with h5part.H5PartFile(path) as f:
        assert f.num_steps() == 1
        f.set_step(0)
        assert f.num_particles() == 777
        # on-disk types as the reference's H5PartType / writeH5PartField choose them
        assert f.field_info("x") == (h5part.F64, 777) and f.field_info("h") == (h5part.F32, 777)
        assert f.field_info("id") == (h5part.I64, 777) and f.field_info("rung") == (h5part.I8, 777)
        assert f.attrib_info("ng0") == (h5part.I32, 1) and f.attrib_info("iteration") == (h5part.I64, 1)
        assert f.attrib_info("box") == (h5part.F64, 6) and f.attrib_info("boundaryType") == (h5part.I8, 3)
        assert f.attrib_info("muiConst") == (h5part.F32, 1) and f.attrib_info("ts::dt_m1") == (h5part.F32, 4)
        with pytest.raises(KeyError):
            f.read_field("nope")


@ref_only
def test_reference_reads_our_file(tmp_path):
    L = ref_lib()
    path = str(tmp_path / "ours.h5")
    st, at = sample_state(1000), sample_attributes()
    h5part.write_step(path, st, at, mode="w")
    st2 = sample_state(1000, seed=2)
    h5part.write_step(path, st2, sample_attributes(13), mode="a")  # Step#1
    bp = path.encode()
    assert L.ref_h5_num_particles(bp, -1) == 1000, L.ref_h5_last_error()
    buf = C.create_string_buffer(4096)
    assert L.ref_h5_step_attributes(bp, 0, buf, 4096) == 0, L.ref_h5_last_error()
    names = set(buf.value.decode().split())
    assert set(sx.ATTRIBUTE_NAMES) <= names
    for k, v in at.items():
        v = np.atleast_1d(np.asarray(v))
        out = np.zeros_like(v)
        rc = L.ref_h5_read_attribute(bp, 0, k.encode(), IOTYPE[v.dtype], out.ctypes.data, v.size)
        assert rc == 0, (k, L.ref_h5_last_error())
        assert np.array_equal(out, v), k
    it = np.zeros(1, np.uint64)
    assert L.ref_h5_read_attribute(bp, -1, b"iteration", 7, it.ctypes.data, 1) == 0 and it[0] == 13
    for step, state in ((0, st), (-1, st2)):
        for k, v in state.items():
            out = np.zeros_like(v)
            assert L.ref_h5_read_field(bp, step, k.encode(), IOTYPE[v.dtype], out.ctypes.data) == 0, k
            assert np.array_equal(out, v), (step, k)


@ref_only
def test_we_read_reference_file(tmp_path):
    L = ref_lib()
    L.ref_h5_write_step.argtypes = [C.c_char_p, C.c_uint64, C.c_int, C.POINTER(C.c_char_p), C.POINTER(C.c_int),
                                    C.POINTER(C.c_void_p), C.c_int, C.POINTER(C.c_char_p), C.POINTER(C.c_int),
                                    C.POINTER(C.c_void_p), C.POINTER(C.c_int64)]
    path = str(tmp_path / "ref.h5")
    n = 513
    st, at = sample_state(n, seed=4), sample_attributes(21)
    keep = []

    def arrays(d):
        names = (C.c_char_p * len(d))(*[k.encode() for k in d])
        vals = [np.ascontiguousarray(np.atleast_1d(np.asarray(v))) for v in d.values()]
        keep.extend(vals)
        types = (C.c_int * len(d))(*[IOTYPE[v.dtype] for v in vals])
        ptrs = (C.c_void_p * len(d))(*[v.ctypes.data for v in vals])
        counts = (C.c_int64 * len(d))(*[v.size for v in vals])
        return names, types, ptrs, counts

    fn, ft, fp, _ = arrays(st)
    an, aty, ap, ac = arrays(at)
    for _ in range(2):  # two steps: the writer appends to an existing file
        rc = L.ref_h5_write_step(path.encode(), n, len(st), fn, ft, fp, len(at), an, aty, ap, ac)
        assert rc == 0, L.ref_h5_last_error()
    with h5part.H5PartFile(path) as f:
        assert f.num_steps() == 2
        f.set_step(1)
        assert f.num_particles() == n
        assert f.field_info("id") == (h5part.I64, n) and f.field_info("rung") == (h5part.I8, n)
        assert f.attrib_info("boundaryType") == (h5part.I8, 3) and f.attrib_info("ng0") == (h5part.I32, 1)
    got, ga = h5part.read_step(path, {k: v.dtype for k, v in st.items()},
                               {k: np.asarray(v).dtype for k, v in at.items()}, step=1)
    for k in st:
        assert np.array_equal(got[k], st[k]), k
    for k in at:
        assert np.array_equal(np.asarray(ga[k]), np.asarray(at[k])), k
