// TEST INFRASTRUCTURE ONLY -- the reference's own H5Part writer and reader (main/src/io/ifile_io_hdf5.cpp over
// extern/h5part/H5Part.c, both compiled from /root/reference by oracle/Makefile into oracle/_ref/libh5part_ref.so),
// driven through a C ABI so tests/test_h5part.py can cross-check sphexa_amd.h5part against them:
//   files written by libsphexa_h5part.so are read by the reference's H5PartReader, and files written by the
//   reference's H5PartWriter are read by libsphexa_h5part.so.
// No reference source is copied here; this file only calls makeH5PartWriter / makeH5PartReader (ifile_io_impl.h).
#include <mpi.h>

#include <cstdint>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "ifile_io_impl.h"

namespace
{

void mpiInit()
{
    int on = 0;
    MPI_Initialized(&on);
    if (!on) MPI_Init(nullptr, nullptr);
}

// type codes = the position in sphexa::IO::Types (ifile_io.hpp:46): double, float, char, uint8_t, int, int64_t,
// unsigned, uint64_t
template<class F>
void withType(int t, void* p, F&& f)
{
    switch (t)
    {
        case 0: f(static_cast<double*>(p)); break;
        case 1: f(static_cast<float*>(p)); break;
        case 2: f(static_cast<char*>(p)); break;
        case 3: f(static_cast<uint8_t*>(p)); break;
        case 4: f(static_cast<int*>(p)); break;
        case 5: f(static_cast<int64_t*>(p)); break;
        case 6: f(static_cast<unsigned*>(p)); break;
        case 7: f(static_cast<uint64_t*>(p)); break;
        default: throw std::runtime_error("bad type code");
    }
}

thread_local std::string lastError;

} // namespace

extern "C"
{
    const char* ref_h5_last_error() { return lastError.c_str(); }

    //! one step through H5PartWriter: addStep, stepAttribute (each), writeField (each), closeStep
    int ref_h5_write_step(const char* path, uint64_t n, int nf, const char** fnames, const int* ftypes,
                          void* const* fdata, int na, const char** anames, const int* atypes, void* const* adata,
                          const int64_t* acounts)
    {
        try
        {
            mpiInit();
            auto w = sphexa::makeH5PartWriter(MPI_COMM_WORLD);
            w->addStep(0, n, path);
            for (int k = 0; k < na; ++k)
                withType(atypes[k], adata[k], [&](auto* p) { w->stepAttribute(anames[k], p, acounts[k]); });
            for (int k = 0; k < nf; ++k)
                withType(ftypes[k], fdata[k], [&](auto* p) { w->writeField(fnames[k], p, k); });
            w->closeStep();
            return 0;
        }
        catch (const std::exception& e)
        {
            lastError = e.what();
            return -1;
        }
    }

    //! H5PartReader::setStep (independent mode) + localNumParticles
    int64_t ref_h5_num_particles(const char* path, int step)
    {
        try
        {
            mpiInit();
            auto r = sphexa::makeH5PartReader(MPI_COMM_WORLD);
            r->setStep(path, step, sphexa::FileMode::independent);
            int64_t n = (int64_t)r->localNumParticles();
            r->closeStep();
            return n;
        }
        catch (const std::exception& e)
        {
            lastError = e.what();
            return -1;
        }
    }

    //! the step attribute names, '\n'-separated into buf
    int ref_h5_step_attributes(const char* path, int step, char* buf, int cap)
    {
        try
        {
            mpiInit();
            auto r = sphexa::makeH5PartReader(MPI_COMM_WORLD);
            r->setStep(path, step, sphexa::FileMode::independent);
            std::string all;
            for (auto& s : r->stepAttributes())
                all += s + "\n";
            r->closeStep();
            if ((int)all.size() + 1 > cap) return -2;
            std::memcpy(buf, all.c_str(), all.size() + 1);
            return 0;
        }
        catch (const std::exception& e)
        {
            lastError = e.what();
            return -1;
        }
    }

    //! stepAttribute(key, typed buffer, size) of the reader: the type checks of readAttribute apply
    int ref_h5_read_attribute(const char* path, int step, const char* key, int type, void* out, int64_t count)
    {
        try
        {
            mpiInit();
            auto r = sphexa::makeH5PartReader(MPI_COMM_WORLD);
            r->setStep(path, step, sphexa::FileMode::independent);
            if (r->stepAttributeSize(key) != count) throw std::runtime_error("attribute size differs");
            withType(type, out, [&](auto* p) { r->stepAttribute(key, p, count); });
            r->closeStep();
            return 0;
        }
        catch (const std::exception& e)
        {
            lastError = e.what();
            return -1;
        }
    }

    int ref_h5_read_field(const char* path, int step, const char* key, int type, void* out)
    {
        try
        {
            mpiInit();
            auto r = sphexa::makeH5PartReader(MPI_COMM_WORLD);
            r->setStep(path, step, sphexa::FileMode::independent);
            withType(type, out, [&](auto* p) { r->readField(key, p); });
            r->closeStep();
            return 0;
        }
        catch (const std::exception& e)
        {
            lastError = e.what();
            return -1;
        }
    }
}
