/*! @file sphexa_h5part.h
 * @brief C-ABI of libsphexa_h5part.so: restart / dump files in the reference's H5Part layout, serial HDF5.
 *
 * Replaces the reference's H5PartWriter / H5PartReader (main/src/io/ifile_io_hdf5.cpp:40-118, :141-300, over
 * extern/h5part/H5Part.c and main/src/io/h5part_wrapper.hpp) for one rank.  Layout, as H5Part writes it:
 *   - one HDF5 file; step k is the root group "Step#k" (H5Part.c:607-627, stepno width 0);
 *   - each field a 1-D dataset of numParticles elements in the step group, native type (H5Part.c:925-1000):
 *     f64 -> H5T_NATIVE_DOUBLE, f32 -> H5T_NATIVE_FLOAT, u8/char -> H5T_NATIVE_INT8, i32/u32 -> H5T_NATIVE_INT32,
 *     i64/u64 -> H5T_NATIVE_INT64 (h5part_wrapper.hpp:280-340);
 *   - step attributes on the step group, file attributes on "/", each a 1-D simple dataspace of `count` elements
 *     (H5Part.c:1325-1380) with H5PartType (h5part_wrapper.hpp:50-95): char/u8 -> H5T_NATIVE_CHAR, others as above;
 *   - the number of particles of a step is the extent of its first dataset (H5Part.c:2476-2560).
 * ParticlesData::loadOrStoreAttributes (sph/particles_data.hpp:141-193) and Box::loadOrStore (sfc/box.hpp:167-175)
 * decide the attribute names and types; sphexa_amd/h5part.py writes and reads them.
 *
 * Type codes of this ABI: SX_H5_F64, SX_H5_F32, SX_H5_I8 (char / uint8), SX_H5_I32 (int / unsigned),
 * SX_H5_I64 (int64 / uint64).  Every function returns 0 on success, a negative SX_H5_ERR_* otherwise.
 */
#ifndef SPHEXA_H5PART_H
#define SPHEXA_H5PART_H

#include <stdint.h>

#ifdef __cplusplus
extern "C"
{
#endif

enum
{
    SX_H5_F64 = 0,
    SX_H5_F32 = 1,
    SX_H5_I8  = 2,
    SX_H5_I32 = 3,
    SX_H5_I64 = 4,
};

enum
{
    SX_H5_OK        = 0,
    SX_H5_ERR_ARG   = -1, /* bad handle, mode, type code or size */
    SX_H5_ERR_IO    = -2, /* an HDF5 call failed (file, group, dataset or attribute) */
    SX_H5_ERR_NOENT = -3, /* no such step, field or attribute */
};

typedef struct sx_h5file sx_h5file;

/*! mode 0 = read, 1 = write (truncate), 2 = append (open read-write, create if missing): H5PART_READ / _WRITE /
 *  _APPEND of H5PartOpenFile (the writer appends when the file exists, ifile_io_hdf5.cpp:59-62) */
int     sx_h5_open(sx_h5file** f, const char* path, int mode);
int     sx_h5_close(sx_h5file* f);
/*! number of "Step#" groups (H5PartGetNumSteps) */
int64_t sx_h5_num_steps(sx_h5file* f);
/*! writing: create step numSteps and make it current (H5PartSetStep + H5PartSetNumParticles, addStep :51-72) */
int     sx_h5_add_step(sx_h5file* f, uint64_t numParticles);
/*! reading: make step `step` current (negative: the last step, H5PartReader::setStep :157-188) */
int     sx_h5_set_step(sx_h5file* f, int64_t step);
/*! particles of the current step (H5PartGetNumParticles) */
int64_t sx_h5_num_particles(sx_h5file* f);
/*! field datasets of the current step */
int     sx_h5_write_field(sx_h5file* f, const char* name, int type, const void* data);
int     sx_h5_read_field(sx_h5file* f, const char* name, int type, void* data);
int     sx_h5_field_info(sx_h5file* f, const char* name, int* type, uint64_t* count);
/*! attributes: scope 0 = the current step's group, 1 = the file ("/") */
int     sx_h5_write_attrib(sx_h5file* f, int scope, const char* name, int type, const void* data, uint64_t count);
int     sx_h5_num_attribs(sx_h5file* f, int scope);
/*! name (NUL-terminated, truncated to cap) of attribute `index` in name order (H5_INDEX_NAME, as H5Aopen_idx) */
int     sx_h5_attrib_name(sx_h5file* f, int scope, int index, char* name, int cap);
int     sx_h5_attrib_info(sx_h5file* f, int scope, const char* name, int* type, uint64_t* count);
/*! read into a buffer of `count` elements of `type` (HDF5 converts; count must equal the stored size, as
 *  readAttribute requires, h5part_wrapper.hpp:177-183) */
int     sx_h5_read_attrib(sx_h5file* f, int scope, const char* name, int type, void* data, uint64_t count);

#ifdef __cplusplus
}
#endif

#endif
