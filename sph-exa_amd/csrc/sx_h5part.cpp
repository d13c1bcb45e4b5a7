/*! @file sx_h5part.cpp
 * @brief H5Part-layout files over serial HDF5 (include/sphexa_h5part.h): the reference's restart/dump format.
 *
 * The reference writes through H5Part (extern/h5part/H5Part.c) behind IFileWriter / IFileReader
 * (main/src/io/ifile_io_hdf5.cpp).  This is a direct HDF5 implementation of the same on-disk layout for one rank:
 * "Step#k" groups, one 1-D native-typed dataset per field, attributes as 1-D simple dataspaces.  Files written here
 * are read by the reference's H5PartReader and vice versa (tests/test_h5part.py, against oracle/_ref's build of
 * H5Part.c + ifile_io_hdf5.cpp).  Host code only: the restart path copies device fields to the host first.
 */
#include <hdf5.h>

#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/sphexa_h5part.h"

struct sx_h5file
{
    hid_t    file{-1};
    hid_t    step{-1}; // current step group
    bool     writable{false};
    uint64_t numParticles{0}; // of the step being written
};

namespace
{

hid_t memType(int t)
{
    switch (t)
    {
        case SX_H5_F64: return H5T_NATIVE_DOUBLE;
        case SX_H5_F32: return H5T_NATIVE_FLOAT;
        case SX_H5_I8: return H5T_NATIVE_INT8;
        case SX_H5_I32: return H5T_NATIVE_INT32;
        case SX_H5_I64: return H5T_NATIVE_INT64;
        default: return -1;
    }
}

//! attributes of char-like type are H5PART_CHAR = H5T_NATIVE_CHAR (h5part_wrapper.hpp:62-72)
hid_t attribType(int t) { return t == SX_H5_I8 ? H5T_NATIVE_CHAR : memType(t); }

//! type code of a stored (file) type: class + size, as H5Part normalises it (_H5Part_normalize_h5_type)
int codeOf(hid_t ftype)
{
    const H5T_class_t cls = H5Tget_class(ftype);
    const size_t      sz  = H5Tget_size(ftype);
    if (cls == H5T_FLOAT) return sz == 8 ? SX_H5_F64 : sz == 4 ? SX_H5_F32 : -1;
    if (cls == H5T_INTEGER) return sz == 1 ? SX_H5_I8 : sz == 4 ? SX_H5_I32 : sz == 8 ? SX_H5_I64 : -1;
    return -1;
}

std::string stepName(int64_t k) { return "Step#" + std::to_string(k); }

herr_t countSteps(hid_t, const char* name, const H5L_info_t*, void* op)
{
    if (std::strncmp(name, "Step#", 5) == 0) ++*static_cast<int64_t*>(op);
    return 0;
}

//! the first dataset of a group (H5Part takes the particle count from it)
herr_t firstDataset(hid_t g, const char* name, const H5L_info_t*, void* op)
{
    H5O_info_t info;
    if (H5Oget_info_by_name2(g, name, &info, H5O_INFO_BASIC, H5P_DEFAULT) < 0) return -1;
    if (info.type != H5O_TYPE_DATASET) return 0;
    *static_cast<std::string*>(op) = name;
    return 1;
}

hid_t scopeId(sx_h5file* f, int scope) { return scope == 1 ? f->file : f->step; }

void closeStep(sx_h5file* f)
{
    if (f->step >= 0) H5Gclose(f->step);
    f->step = -1;
}

} // namespace

extern "C"
{
    int sx_h5_open(sx_h5file** out, const char* path, int mode)
    {
        if (!out || !path || mode < 0 || mode > 2) return SX_H5_ERR_ARG;
        H5Eset_auto2(H5E_DEFAULT, nullptr, nullptr); // errors are return codes here, not stderr
        auto* f = new sx_h5file;
        if (mode == 0) f->file = H5Fopen(path, H5F_ACC_RDONLY, H5P_DEFAULT);
        else if (mode == 1) f->file = H5Fcreate(path, H5F_ACC_TRUNC, H5P_DEFAULT, H5P_DEFAULT);
        else
        {
            FILE* probe = std::fopen(path, "rb");
            if (probe)
            {
                std::fclose(probe);
                f->file = H5Fopen(path, H5F_ACC_RDWR, H5P_DEFAULT);
            }
            else f->file = H5Fcreate(path, H5F_ACC_TRUNC, H5P_DEFAULT, H5P_DEFAULT);
        }
        if (f->file < 0)
        {
            delete f;
            return mode == 0 ? SX_H5_ERR_NOENT : SX_H5_ERR_IO;
        }
        f->writable = mode != 0;
        *out        = f;
        return SX_H5_OK;
    }

    int sx_h5_close(sx_h5file* f)
    {
        if (!f) return SX_H5_ERR_ARG;
        closeStep(f);
        herr_t e = f->file >= 0 ? H5Fclose(f->file) : 0;
        delete f;
        return e < 0 ? SX_H5_ERR_IO : SX_H5_OK;
    }

    int64_t sx_h5_num_steps(sx_h5file* f)
    {
        if (!f) return SX_H5_ERR_ARG;
        int64_t n = 0;
        if (H5Literate(f->file, H5_INDEX_NAME, H5_ITER_INC, nullptr, countSteps, &n) < 0) return SX_H5_ERR_IO;
        return n;
    }

    int sx_h5_add_step(sx_h5file* f, uint64_t numParticles)
    {
        if (!f || !f->writable) return SX_H5_ERR_ARG;
        int64_t k = sx_h5_num_steps(f);
        if (k < 0) return (int)k;
        closeStep(f);
        f->step = H5Gcreate2(f->file, stepName(k).c_str(), H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT);
        if (f->step < 0) return SX_H5_ERR_IO;
        f->numParticles = numParticles;
        return SX_H5_OK;
    }

    int sx_h5_set_step(sx_h5file* f, int64_t step)
    {
        if (!f) return SX_H5_ERR_ARG;
        int64_t n = sx_h5_num_steps(f);
        if (n < 0) return (int)n;
        if (step < 0) step = n - 1;
        if (step < 0 || step >= n) return SX_H5_ERR_NOENT;
        closeStep(f);
        f->step = H5Gopen2(f->file, stepName(step).c_str(), H5P_DEFAULT);
        if (f->step < 0) return SX_H5_ERR_NOENT;
        f->numParticles = 0;
        return SX_H5_OK;
    }

    int64_t sx_h5_num_particles(sx_h5file* f)
    {
        if (!f || f->step < 0) return SX_H5_ERR_ARG;
        std::string first;
        if (H5Literate(f->step, H5_INDEX_NAME, H5_ITER_INC, nullptr, firstDataset, &first) < 0) return SX_H5_ERR_IO;
        if (first.empty()) return (int64_t)f->numParticles; // nothing written yet: the count set with the step
        hid_t d = H5Dopen2(f->step, first.c_str(), H5P_DEFAULT);
        if (d < 0) return SX_H5_ERR_IO;
        hid_t   sp = H5Dget_space(d);
        hssize_t n = H5Sget_simple_extent_npoints(sp);
        H5Sclose(sp);
        H5Dclose(d);
        return n < 0 ? SX_H5_ERR_IO : (int64_t)n;
    }

    int sx_h5_write_field(sx_h5file* f, const char* name, int type, const void* data)
    {
        if (!f || !f->writable || f->step < 0 || !name) return SX_H5_ERR_ARG;
        hid_t mt = memType(type);
        if (mt < 0 || (!data && f->numParticles)) return SX_H5_ERR_ARG;
        hsize_t dim = f->numParticles;
        hid_t   sp  = H5Screate_simple(1, &dim, nullptr);
        if (sp < 0) return SX_H5_ERR_IO;
        hid_t d = H5Dcreate2(f->step, name, mt, sp, H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT);
        int   rc = SX_H5_OK;
        if (d < 0) rc = SX_H5_ERR_IO;
        else
        {
            if (dim && H5Dwrite(d, mt, H5S_ALL, H5S_ALL, H5P_DEFAULT, data) < 0) rc = SX_H5_ERR_IO;
            H5Dclose(d);
        }
        H5Sclose(sp);
        return rc;
    }

    int sx_h5_field_info(sx_h5file* f, const char* name, int* type, uint64_t* count)
    {
        if (!f || f->step < 0 || !name) return SX_H5_ERR_ARG;
        if (H5Lexists(f->step, name, H5P_DEFAULT) <= 0) return SX_H5_ERR_NOENT;
        hid_t d = H5Dopen2(f->step, name, H5P_DEFAULT);
        if (d < 0) return SX_H5_ERR_NOENT;
        hid_t    ft = H5Dget_type(d), sp = H5Dget_space(d);
        hssize_t n  = H5Sget_simple_extent_npoints(sp);
        if (type) *type = codeOf(ft);
        if (count) *count = (uint64_t)n;
        H5Tclose(ft);
        H5Sclose(sp);
        H5Dclose(d);
        return SX_H5_OK;
    }

    int sx_h5_read_field(sx_h5file* f, const char* name, int type, void* data)
    {
        if (!f || f->step < 0 || !name) return SX_H5_ERR_ARG;
        hid_t mt = memType(type);
        if (mt < 0) return SX_H5_ERR_ARG;
        if (H5Lexists(f->step, name, H5P_DEFAULT) <= 0) return SX_H5_ERR_NOENT;
        hid_t d = H5Dopen2(f->step, name, H5P_DEFAULT);
        if (d < 0) return SX_H5_ERR_NOENT;
        int rc = H5Dread(d, mt, H5S_ALL, H5S_ALL, H5P_DEFAULT, data) < 0 ? SX_H5_ERR_IO : SX_H5_OK;
        H5Dclose(d);
        return rc;
    }

    int sx_h5_write_attrib(sx_h5file* f, int scope, const char* name, int type, const void* data, uint64_t count)
    {
        if (!f || !f->writable || !name || !data || count == 0) return SX_H5_ERR_ARG;
        hid_t loc = scopeId(f, scope);
        hid_t at  = attribType(type);
        if (loc < 0 || at < 0) return SX_H5_ERR_ARG;
        hsize_t dim = count;
        hid_t   sp  = H5Screate_simple(1, &dim, nullptr);
        if (sp < 0) return SX_H5_ERR_IO;
        if (H5Aexists(loc, name) > 0) H5Adelete(loc, name); // re-writing an attribute replaces it
        hid_t a  = H5Acreate2(loc, name, at, sp, H5P_DEFAULT, H5P_DEFAULT);
        int   rc = SX_H5_OK;
        if (a < 0) rc = SX_H5_ERR_IO;
        else
        {
            if (H5Awrite(a, at, data) < 0) rc = SX_H5_ERR_IO;
            H5Aclose(a);
        }
        H5Sclose(sp);
        return rc;
    }

    int sx_h5_num_attribs(sx_h5file* f, int scope)
    {
        if (!f) return SX_H5_ERR_ARG;
        hid_t loc = scopeId(f, scope);
        if (loc < 0) return SX_H5_ERR_ARG;
        H5O_info_t info;
        if (H5Oget_info2(loc, &info, H5O_INFO_NUM_ATTRS) < 0) return SX_H5_ERR_IO;
        return (int)info.num_attrs;
    }

    int sx_h5_attrib_name(sx_h5file* f, int scope, int index, char* name, int cap)
    {
        if (!f || !name || cap < 1) return SX_H5_ERR_ARG;
        hid_t loc = scopeId(f, scope);
        if (loc < 0) return SX_H5_ERR_ARG;
        ssize_t n = H5Aget_name_by_idx(loc, ".", H5_INDEX_NAME, H5_ITER_INC, (hsize_t)index, name, (size_t)cap,
                                       H5P_DEFAULT);
        return n < 0 ? SX_H5_ERR_NOENT : SX_H5_OK;
    }

    int sx_h5_attrib_info(sx_h5file* f, int scope, const char* name, int* type, uint64_t* count)
    {
        if (!f || !name) return SX_H5_ERR_ARG;
        hid_t loc = scopeId(f, scope);
        if (loc < 0) return SX_H5_ERR_ARG;
        if (H5Aexists(loc, name) <= 0) return SX_H5_ERR_NOENT;
        hid_t a = H5Aopen(loc, name, H5P_DEFAULT);
        if (a < 0) return SX_H5_ERR_IO;
        hid_t    ft = H5Aget_type(a), sp = H5Aget_space(a);
        hssize_t n  = H5Sget_simple_extent_npoints(sp);
        if (type) *type = codeOf(ft);
        if (count) *count = (uint64_t)n;
        H5Tclose(ft);
        H5Sclose(sp);
        H5Aclose(a);
        return SX_H5_OK;
    }

    int sx_h5_read_attrib(sx_h5file* f, int scope, const char* name, int type, void* data, uint64_t count)
    {
        uint64_t stored = 0;
        if (int e = sx_h5_attrib_info(f, scope, name, nullptr, &stored)) return e;
        hid_t mt = memType(type);
        if (mt < 0 || !data || stored != count) return SX_H5_ERR_ARG;
        hid_t a  = H5Aopen(scopeId(f, scope), name, H5P_DEFAULT);
        int   rc = H5Aread(a, mt, data) < 0 ? SX_H5_ERR_IO : SX_H5_OK;
        H5Aclose(a);
        return rc;
    }
}
