// libtmh5.so — the HDF5 files of the illumination path, without h5py.
//
// Layouts (unchanged from the reference):
//   illumstats_file_{id}.h5  (tmlib/models/file.py:440-456 IllumstatsFile.put via
//                             tmlib/writers.py:322-389 DatasetWriter.write)
//     /mean                f64 [H, W]   contiguous, uncompressed
//     /std                 f64 [H, W]
//     /percentiles/keys    f64 [Q]
//     /percentiles/values  i64 [Q]
//   channel_image_file_{id}.h5 (tmlib/models/file.py:353-363 ChannelImageFile.put,
//                               read at :322-351 via tmlib/readers.py:367-389)
//     /array               u8/u16 [H, W]  gzip-compressed, chunked
//
// Error convention as libtmhip: 0 ok, negative errno-style code on failure,
// message in tmh5_last_error().
#include <hdf5.h>

#include <cstdint>
#include <cstring>
#include <string>

#include "../../include/tmh5.h"

namespace {

thread_local std::string g_err;

struct H5Err {
  int code;
  std::string msg;
};

struct Hid {  // closes an HDF5 identifier with the right function
  hid_t id = -1;
  herr_t (*close)(hid_t) = nullptr;
  Hid(hid_t i, herr_t (*c)(hid_t)) : id(i), close(c) {
    if (id < 0) throw H5Err{-5, "HDF5 call failed"};
  }
  ~Hid() {
    if (id >= 0 && close) close(id);
  }
  operator hid_t() const { return id; }
};

template <typename F>
int guard(F&& f) {
  try {
    f();
    return 0;
  } catch (const H5Err& e) {
    g_err = e.msg;
    return e.code;
  } catch (...) {
    g_err = "unknown error";
    return -5;
  }
}

void silence() { H5Eset_auto2(H5E_DEFAULT, nullptr, nullptr); }

void write_ds(hid_t file, const char* name, hid_t ftype, hid_t mtype, int rank,
              const hsize_t* dims, const void* data, hid_t dcpl = H5P_DEFAULT) {
  Hid lcpl(H5Pcreate(H5P_LINK_CREATE), H5Pclose);
  H5Pset_create_intermediate_group(lcpl, 1);
  Hid sp(H5Screate_simple(rank, dims, nullptr), H5Sclose);
  Hid ds(H5Dcreate2(file, name, ftype, sp, lcpl, dcpl, H5P_DEFAULT), H5Dclose);
  if (H5Dwrite(ds, mtype, H5S_ALL, H5S_ALL, H5P_DEFAULT, data) < 0)
    throw H5Err{-5, std::string("writing ") + name + " failed"};
}

// dims of a dataset; returns rank
int ds_dims(hid_t file, const char* name, hsize_t* dims, int max_rank) {
  if (H5Lexists(file, name, H5P_DEFAULT) <= 0) throw H5Err{-2, std::string("Dataset does not exist: ") + name};
  Hid ds(H5Dopen2(file, name, H5P_DEFAULT), H5Dclose);
  Hid sp(H5Dget_space(ds), H5Sclose);
  int r = H5Sget_simple_extent_ndims(sp);
  if (r < 0 || r > max_rank) throw H5Err{-22, std::string("unexpected rank of ") + name};
  H5Sget_simple_extent_dims(sp, dims, nullptr);
  return r;
}

void read_ds(hid_t file, const char* name, hid_t mtype, void* out) {
  Hid ds(H5Dopen2(file, name, H5P_DEFAULT), H5Dclose);
  if (H5Dread(ds, mtype, H5S_ALL, H5S_ALL, H5P_DEFAULT, out) < 0)
    throw H5Err{-5, std::string("reading ") + name + " failed"};
}

}  // namespace

extern "C" {

const char* tmh5_last_error(void) { return g_err.c_str(); }

int tmh5_write_illumstats(const char* path, int height, int width, const double* mean,
                          const double* std_, int64_t n_quantiles, const double* keys,
                          const int64_t* values) {
  return guard([&] {
    silence();
    if (!path || !mean || !std_ || height <= 0 || width <= 0 || n_quantiles < 0 ||
        (n_quantiles && (!keys || !values)))
      throw H5Err{-22, "bad arguments"};
    Hid f(H5Fcreate(path, H5F_ACC_TRUNC, H5P_DEFAULT, H5P_DEFAULT), H5Fclose);
    const hsize_t d2[2] = {(hsize_t)height, (hsize_t)width};
    const hsize_t d1[1] = {(hsize_t)n_quantiles};
    write_ds(f, "mean", H5T_IEEE_F64LE, H5T_NATIVE_DOUBLE, 2, d2, mean);
    write_ds(f, "std", H5T_IEEE_F64LE, H5T_NATIVE_DOUBLE, 2, d2, std_);
    write_ds(f, "/percentiles/keys", H5T_IEEE_F64LE, H5T_NATIVE_DOUBLE, 1, d1, keys);
    write_ds(f, "/percentiles/values", H5T_STD_I64LE, H5T_NATIVE_INT64, 1, d1, values);
  });
}

int tmh5_illumstats_shape(const char* path, int* height, int* width, int64_t* n_quantiles) {
  return guard([&] {
    silence();
    if (!path || !height || !width || !n_quantiles) throw H5Err{-22, "bad arguments"};
    Hid f(H5Fopen(path, H5F_ACC_RDONLY, H5P_DEFAULT), H5Fclose);
    hsize_t d[2] = {0, 0};
    if (ds_dims(f, "mean", d, 2) != 2) throw H5Err{-22, "/mean is not 2-D"};
    *height = (int)d[0];
    *width = (int)d[1];
    hsize_t q[1] = {0};
    ds_dims(f, "/percentiles/keys", q, 1);
    *n_quantiles = (int64_t)q[0];
  });
}

int tmh5_read_illumstats(const char* path, double* mean, double* std_, double* keys,
                         int64_t* values) {
  return guard([&] {
    silence();
    if (!path) throw H5Err{-22, "bad arguments"};
    Hid f(H5Fopen(path, H5F_ACC_RDONLY, H5P_DEFAULT), H5Fclose);
    if (mean) read_ds(f, "mean", H5T_NATIVE_DOUBLE, mean);
    if (std_) read_ds(f, "std", H5T_NATIVE_DOUBLE, std_);
    if (keys) read_ds(f, "/percentiles/keys", H5T_NATIVE_DOUBLE, keys);
    if (values) read_ds(f, "/percentiles/values", H5T_NATIVE_INT64, values);
  });
}

int tmh5_write_channel_image(const char* path, int height, int width, int bits, const void* data,
                             int gzip_level) {
  return guard([&] {
    silence();
    if (!path || !data || height <= 0 || width <= 0 || (bits != 8 && bits != 16))
      throw H5Err{-22, "bad arguments"};
    Hid f(H5Fcreate(path, H5F_ACC_TRUNC, H5P_DEFAULT, H5P_DEFAULT), H5Fclose);
    const hsize_t d2[2] = {(hsize_t)height, (hsize_t)width};
    Hid dcpl(H5Pcreate(H5P_DATASET_CREATE), H5Pclose);
    if (gzip_level >= 0) {
      // chunk of whole rows, ~256 KiB, like h5py's automatic chunking scale
      const hsize_t row_bytes = (hsize_t)width * (bits / 8);
      hsize_t rows = row_bytes ? (262144 + row_bytes - 1) / row_bytes : 1;
      if (rows > (hsize_t)height) rows = height;
      const hsize_t chunk[2] = {rows, (hsize_t)width};
      H5Pset_chunk(dcpl, 2, chunk);
      H5Pset_deflate(dcpl, (unsigned)(gzip_level > 9 ? 9 : gzip_level));
    }
    write_ds(f, "array", bits == 8 ? H5T_STD_U8LE : H5T_STD_U16LE,
             bits == 8 ? H5T_NATIVE_UINT8 : H5T_NATIVE_UINT16, 2, d2, data, dcpl);
  });
}

int tmh5_channel_image_shape(const char* path, int* height, int* width, int* bits) {
  return guard([&] {
    silence();
    if (!path || !height || !width || !bits) throw H5Err{-22, "bad arguments"};
    Hid f(H5Fopen(path, H5F_ACC_RDONLY, H5P_DEFAULT), H5Fclose);
    hsize_t d[2] = {0, 0};
    if (ds_dims(f, "array", d, 2) != 2) throw H5Err{-22, "/array is not 2-D"};
    Hid ds(H5Dopen2(f, "array", H5P_DEFAULT), H5Dclose);
    Hid t(H5Dget_type(ds), H5Tclose);
    if (H5Tget_class(t) != H5T_INTEGER || H5Tget_sign(t) != H5T_SGN_NONE)
      throw H5Err{-22, "/array must hold unsigned integers"};
    *bits = (int)H5Tget_size(t) * 8;
    if (*bits != 8 && *bits != 16) throw H5Err{-22, "/array must be uint8 or uint16"};
    *height = (int)d[0];
    *width = (int)d[1];
  });
}

int tmh5_read_channel_image(const char* path, void* out) {
  return guard([&] {
    silence();
    if (!path || !out) throw H5Err{-22, "bad arguments"};
    Hid f(H5Fopen(path, H5F_ACC_RDONLY, H5P_DEFAULT), H5Fclose);
    Hid ds(H5Dopen2(f, "array", H5P_DEFAULT), H5Dclose);
    Hid t(H5Dget_type(ds), H5Tclose);
    const hid_t mtype = H5Tget_size(t) == 1 ? H5T_NATIVE_UINT8 : H5T_NATIVE_UINT16;
    if (H5Dread(ds, mtype, H5S_ALL, H5S_ALL, H5P_DEFAULT, out) < 0)
      throw H5Err{-5, "reading /array failed"};
  });
}

}  // extern "C"
