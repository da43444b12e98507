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
#include <zlib.h>

#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <mutex>
#include <thread>
#include <vector>

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
  return tmh5_write_channel_image_chunked(path, height, width, bits, data, gzip_level, 0, 0);
}

int tmh5_write_channel_image_chunked(const char* path, int height, int width, int bits,
                                     const void* data, int gzip_level, int chunk_rows,
                                     int chunk_cols) {
  return guard([&] {
    silence();
    if (!path || !data || height <= 0 || width <= 0 || (bits != 8 && bits != 16) ||
        chunk_rows < 0 || chunk_cols < 0)
      throw H5Err{-22, "bad arguments"};
    Hid f(H5Fcreate(path, H5F_ACC_TRUNC, H5P_DEFAULT, H5P_DEFAULT), H5Fclose);
    const hsize_t d2[2] = {(hsize_t)height, (hsize_t)width};
    Hid dcpl(H5Pcreate(H5P_DATASET_CREATE), H5Pclose);
    if (gzip_level >= 0) {
      // default: chunks of whole rows, ~256 KiB, like h5py's automatic chunking scale
      const hsize_t row_bytes = (hsize_t)width * (bits / 8);
      hsize_t rows = row_bytes ? (262144 + row_bytes - 1) / row_bytes : 1;
      if (rows > (hsize_t)height) rows = height;
      hsize_t chunk[2] = {rows, (hsize_t)width};
      if (chunk_rows > 0) chunk[0] = std::min<hsize_t>(chunk_rows, height);
      if (chunk_cols > 0) chunk[1] = std::min<hsize_t>(chunk_cols, width);
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

// Many channel images at once (the input path is
// bound by gzip inflate, not by the GPU).  libhdf5 serialises every call
// behind its global lock -- including the deflate filter inside H5Dread -- so
// the workers take only the raw compressed chunks from HDF5
// (H5Dget_chunk_info + H5Dread_chunk) and inflate them with zlib in
// parallel, straight into the caller's [n][H][W] buffer.  Datasets that are
// not chunked+deflate-only (contiguous, shuffle, other filters) are read
// with H5Dread instead.  All files must share one shape and dtype.
namespace {

void read_one_parallel(const char* path, uint8_t* out, int height, int width, int esize) {
  std::vector<std::vector<uint8_t>> raw;
  std::vector<std::pair<hsize_t, hsize_t>> offs;
  std::vector<char> stored;  // filter mask: deflate skipped for this chunk
  hsize_t ch[2] = {0, 0};
  {
    Hid f(H5Fopen(path, H5F_ACC_RDONLY, H5P_DEFAULT), H5Fclose);
    Hid ds(H5Dopen2(f, "array", H5P_DEFAULT), H5Dclose);
    Hid t(H5Dget_type(ds), H5Tclose);
    Hid sp(H5Dget_space(ds), H5Sclose);
    hsize_t d[2] = {0, 0};
    if (H5Sget_simple_extent_ndims(sp) != 2) throw H5Err{-22, std::string(path) + ": /array is not 2-D"};
    H5Sget_simple_extent_dims(sp, d, nullptr);
    if ((int)d[0] != height || (int)d[1] != width || (int)H5Tget_size(t) != esize ||
        H5Tget_class(t) != H5T_INTEGER || H5Tget_sign(t) != H5T_SGN_NONE)
      throw H5Err{-22, std::string(path) + ": shape or dtype differs from the first image"};
    Hid dcpl(H5Dget_create_plist(ds), H5Pclose);
    bool direct = H5Pget_layout(dcpl) == H5D_CHUNKED && H5Pget_nfilters(dcpl) == 1 &&
                  H5Tget_order(t) == H5T_ORDER_LE;
    if (direct) {
      unsigned flags = 0, cd[8];
      size_t ncd = 8;
      direct = H5Pget_filter2(dcpl, 0, &flags, &ncd, cd, 0, nullptr, nullptr) == H5Z_FILTER_DEFLATE &&
               H5Pget_chunk(dcpl, 2, ch) == 2;
    }
    if (!direct) {
      const hid_t mtype = esize == 1 ? H5T_NATIVE_UINT8 : H5T_NATIVE_UINT16;
      if (H5Dread(ds, mtype, H5S_ALL, H5S_ALL, H5P_DEFAULT, out) < 0)
        throw H5Err{-5, std::string(path) + ": reading /array failed"};
      return;
    }
    hsize_t nchunks = 0;
    if (H5Dget_num_chunks(ds, sp, &nchunks) < 0) throw H5Err{-5, "H5Dget_num_chunks failed"};
    if (nchunks < (hsize_t)(((d[0] + ch[0] - 1) / ch[0]) * ((d[1] + ch[1] - 1) / ch[1])))
      memset(out, 0, (size_t)height * width * esize);  // unwritten chunks read as fill (0)
    raw.reserve(nchunks);
    offs.reserve(nchunks);
    stored.reserve(nchunks);
    // every chunk of the grid by coordinates (unwritten ones have no address):
    // H5Dget_chunk_info by index walks the chunk index from its start per call
    const hsize_t gr = (d[0] + ch[0] - 1) / ch[0], gc = (d[1] + ch[1] - 1) / ch[1];
    for (hsize_t g = 0; g < gr * gc; ++g) {
      hsize_t coord[2] = {(g / gc) * ch[0], (g % gc) * ch[1]};
      unsigned fmask = 0;
      haddr_t addr = HADDR_UNDEF;
      hsize_t size = 0;
      if (H5Dget_chunk_info_by_coord(ds, coord, &fmask, &addr, &size) < 0)
        throw H5Err{-5, std::string(path) + ": H5Dget_chunk_info_by_coord failed"};
      if (addr == HADDR_UNDEF) continue;  // unwritten: fill value
      const size_t i = raw.size();
      raw.emplace_back();
      offs.emplace_back();
      stored.push_back(0);
      raw[i].resize(size);
      uint32_t fm = 0;
      if (H5Dread_chunk(ds, H5P_DEFAULT, coord, &fm, raw[i].data()) < 0)
        throw H5Err{-5, "H5Dread_chunk failed"};
      stored[i] = (fm & 1u) ? 1 : 0;
      offs[i] = {coord[0], coord[1]};
    }
  }
  // inflate outside the HDF5 lock
  const size_t full = (size_t)(ch[0] * ch[1]) * esize;
  std::vector<uint8_t> buf(full);
  for (size_t i = 0; i < raw.size(); ++i) {
    uLongf len = (uLongf)full;
    const uint8_t* src = buf.data();
    if (stored[i]) {
      if (raw[i].size() != full) throw H5Err{-5, std::string(path) + ": bad unfiltered chunk"};
      src = raw[i].data();
    } else if (uncompress(buf.data(), &len, raw[i].data(), (uLong)raw[i].size()) != Z_OK ||
               len != (uLongf)full) {
      throw H5Err{-5, std::string(path) + ": corrupt deflate chunk"};
    }
    const hsize_t r0 = offs[i].first, c0 = offs[i].second;
    const hsize_t rows = std::min<hsize_t>(ch[0], (hsize_t)height - r0);
    const hsize_t cols = std::min<hsize_t>(ch[1], (hsize_t)width - c0);
    for (hsize_t r = 0; r < rows; ++r)
      memcpy(out + ((r0 + r) * (hsize_t)width + c0) * esize, src + r * ch[1] * esize,
             (size_t)cols * esize);
  }
}

}  // namespace

// Raw chunks for the GPU inflate (tmh_inflate_device): per file, under
// libhdf5's lock, the /array layout checks and every chunk's (coordinates,
// filter mask, file address, size); then the compressed bytes are read with
// pread() by n_threads workers outside the lock, straight into the caller's
// blob.  (H5Dread_chunk would move the bytes under the lock; the addresses
// H5Dget_chunk_info reports are relative to the file's base address, the
// userblock size.)
namespace {

struct FileChunks {
  std::vector<tmh5_chunk> ch;  // src_off relative to the file's first chunk in the blob
  std::vector<int64_t> addr;   // absolute file offset of each chunk
  int64_t bytes = 0;
  // from the HDF5 pass, for the index parse
  uint64_t ub = 0;       // userblock = base address
  uint64_t oh = 0;       // /array's object header address
  hsize_t d[2] = {0, 0};  // dataset extent
  hsize_t n = 0;          // chunks
  bool parsed = false;
};

// Under the HDF5 lock: the /array checks, the chunk count, and where its
// object header is.  The chunk index itself is read by parse_chunk_index
// (outside the lock, in parallel) or, failing that, by chunks_by_hdf5.
void file_header(const char* path, int64_t image, int h, int w, int esize, hsize_t* ch,
                 FileChunks& fc) {
  Hid f(H5Fopen(path, H5F_ACC_RDONLY, H5P_DEFAULT), H5Fclose);
  hsize_t ub = 0;
  {
    Hid fcpl(H5Fget_create_plist(f), H5Pclose);
    H5Pget_userblock(fcpl, &ub);
  }
  Hid ds(H5Dopen2(f, "array", H5P_DEFAULT), H5Dclose);
  Hid t(H5Dget_type(ds), H5Tclose);
  Hid sp(H5Dget_space(ds), H5Sclose);
  hsize_t d[2] = {0, 0};
  if (H5Sget_simple_extent_ndims(sp) != 2) throw H5Err{-22, std::string(path) + ": /array is not 2-D"};
  H5Sget_simple_extent_dims(sp, d, nullptr);
  if ((int)d[0] != h || (int)d[1] != w || (int)H5Tget_size(t) != esize ||
      H5Tget_class(t) != H5T_INTEGER || H5Tget_sign(t) != H5T_SGN_NONE)
    throw H5Err{-22, std::string(path) + ": shape or dtype differs from the first image"};
  Hid dcpl(H5Dget_create_plist(ds), H5Pclose);
  hsize_t c[2] = {0, 0};
  unsigned flags = 0, cd[8];
  size_t ncd = 8;
  if (H5Pget_layout(dcpl) != H5D_CHUNKED || H5Pget_nfilters(dcpl) != 1 ||
      H5Tget_order(t) != H5T_ORDER_LE || H5Pget_chunk(dcpl, 2, c) != 2 ||
      H5Pget_filter2(dcpl, 0, &flags, &ncd, cd, 0, nullptr, nullptr) != H5Z_FILTER_DEFLATE)
    throw H5Err{-95, std::string(path) + ": /array is not chunked with the deflate filter only"};
  if (ch[0] == 0) {
    ch[0] = c[0];
    ch[1] = c[1];
  } else if (c[0] != ch[0] || c[1] != ch[1]) {
    throw H5Err{-95, std::string(path) + ": chunk shape differs from the first image"};
  }
  hsize_t n = 0;
  if (H5Dget_num_chunks(ds, sp, &n) < 0) throw H5Err{-5, "H5Dget_num_chunks failed"};
  if (n != ((d[0] + c[0] - 1) / c[0]) * ((d[1] + c[1] - 1) / c[1]))  // unwritten chunks: fill values
    throw H5Err{-95, std::string(path) + ": /array has unwritten chunks"};
  H5O_info_t oi;
  fc.oh = H5Oget_info2(ds, &oi, H5O_INFO_BASIC) >= 0 ? (uint64_t)oi.addr : 0;
  fc.ub = ub;
  fc.d[0] = d[0];
  fc.d[1] = d[1];
  fc.n = n;
  fc.ch.assign(n, tmh5_chunk{});
  fc.addr.assign(n, 0);
  for (auto& e : fc.ch) e.image = image;
}

// The table from libhdf5, chunk by chunk (any chunk index; ~1.5 us a chunk
// under the lock -- the fallback of parse_chunk_index).
void chunks_by_hdf5(const char* path, int esize, const hsize_t* c, FileChunks& fc) {
  Hid f(H5Fopen(path, H5F_ACC_RDONLY, H5P_DEFAULT), H5Fclose);
  Hid ds(H5Dopen2(f, "array", H5P_DEFAULT), H5Dclose);
  const int64_t raw = (int64_t)(c[0] * c[1]) * esize;
  const hsize_t gc = (fc.d[1] + c[1] - 1) / c[1];
  fc.bytes = 0;
  for (hsize_t i = 0; i < fc.n; ++i) {
    hsize_t coord[2] = {(i / gc) * c[0], (i % gc) * c[1]};
    unsigned fmask = 0;
    haddr_t addr = HADDR_UNDEF;
    hsize_t size = 0;
    if (H5Dget_chunk_info_by_coord(ds, coord, &fmask, &addr, &size) < 0 || addr == HADDR_UNDEF)
      throw H5Err{-5, std::string(path) + ": H5Dget_chunk_info_by_coord failed"};
    tmh5_chunk& e = fc.ch[i];
    e.src_off = fc.bytes;
    e.src_len = (int64_t)size;
    e.raw_len = raw;
    e.row0 = (int32_t)coord[0];
    e.col0 = (int32_t)coord[1];
    e.flags = (fmask & 1u) ? 1 : 0;  // deflate skipped for this chunk: stored
    e.reserved = 0;
    fc.addr[i] = (int64_t)(fc.ub + addr);
    fc.bytes += (int64_t)size;
  }
}

uint64_t le(const uint8_t* p, int n) {
  uint64_t v = 0;
  for (int i = 0; i < n; ++i) v |= (uint64_t)p[i] << (8 * i);
  return v;
}

bool pread_all(int fd, void* dst, size_t n, uint64_t pos) {
  uint8_t* d = static_cast<uint8_t*>(dst);
  while (n > 0) {
    const ssize_t r = pread(fd, d, n, (off_t)pos);
    if (r <= 0) return false;
    d += r;
    pos += (uint64_t)r;
    n -= (size_t)r;
  }
  return true;
}

// The chunk table read straight from the file's bytes, without libhdf5 (so
// outside its lock, one file per worker): the HDF5 file format's version-1
// object header of /array -> its data layout message (version 3, chunked) ->
// the version-1 B-tree of raw data chunks, whose leaf keys hold each chunk's
// size, filter mask and offset and whose children are the chunk addresses.
// This is the layout libhdf5 writes at its default (earliest) format
// bounds, as h5py does for the reference's files.  Anything else (version-2
// object headers, other chunk indexes, 4-byte addresses) returns false and
// the file goes through chunks_by_hdf5.  The result is checked for exactly
// one chunk per grid cell.
bool parse_chunk_index(const char* path, int esize, const hsize_t* c, FileChunks& fc) {
  if (!fc.oh) return false;
  const int fd = open(path, O_RDONLY);
  if (fd < 0) return false;
  struct Close {
    int fd;
    ~Close() { close(fd); }
  } cl{fd};
  uint8_t sb[16];
  if (!pread_all(fd, sb, 16, fc.ub) || memcmp(sb, "\x89HDF\r\n\x1a\n", 8) != 0) return false;
  const int sbv = sb[8];
  const int so = sbv <= 1 ? sb[13] : sb[9], sl = sbv <= 1 ? sb[14] : sb[10];
  if (so != 8 || sl != 8) return false;
  // object header v1: version, reserved, #messages (2), refcount (4), header size (4), pad to 16
  uint8_t oh[16];
  if (!pread_all(fd, oh, 16, fc.ub + fc.oh) || oh[0] != 1) return false;
  const uint64_t nmsg = le(oh + 2, 2);
  std::vector<std::pair<uint64_t, uint64_t>> blocks{{fc.ub + fc.oh + 16, le(oh + 8, 4)}};
  uint64_t bt = 0;
  bool found = false;
  uint64_t seen = 0;
  std::vector<uint8_t> buf;
  for (size_t bi = 0; bi < blocks.size() && !found && seen < nmsg && bi < 64; ++bi) {
    buf.resize(blocks[bi].second);
    if (buf.size() > (1u << 20) || !pread_all(fd, buf.data(), buf.size(), blocks[bi].first))
      return false;
    for (size_t o = 0; o + 8 <= buf.size() && seen < nmsg;) {
      const uint64_t type = le(&buf[o], 2), size = le(&buf[o + 2], 2);
      const uint8_t* m = &buf[o + 8];
      if (o + 8 + size > buf.size()) return false;
      ++seen;
      if (type == 0x10 && size >= 16) {  // continuation
        blocks.push_back({fc.ub + le(m, 8), le(m + 8, 8)});
      } else if (type == 0x08) {  // data layout
        if (size < 3 + 8 + 12 || m[0] != 3 || m[1] != 2 || m[2] != 3) return false;
        if (le(m + 11, 4) != c[0] || le(m + 15, 4) != c[1] || (int)le(m + 19, 4) != esize)
          return false;
        bt = le(m + 3, 8);
        found = true;
        break;
      }
      o += 8 + size;
    }
  }
  if (!found || bt == ~0ull) return false;
  // B-tree v1 (type 1): "TREE", type, level, entries (2), left, right (8 + 8),
  // then key, child, ..., key; key = size (4), filter mask (4), 3 offsets (8 each)
  constexpr size_t kKey = 32;
  const hsize_t gr = (fc.d[0] + c[0] - 1) / c[0], gc = (fc.d[1] + c[1] - 1) / c[1];
  std::vector<char> have(fc.n, 0);
  std::vector<uint64_t> stack{bt};
  const int64_t raw = (int64_t)(c[0] * c[1]) * esize;
  hsize_t got = 0;
  size_t visits = 0;
  while (!stack.empty()) {
    const uint64_t a = stack.back();
    stack.pop_back();
    if (++visits > 4 * fc.n + 64) return false;
    uint8_t hd[24];
    if (!pread_all(fd, hd, 24, fc.ub + a) || memcmp(hd, "TREE", 4) != 0 || hd[4] != 1) return false;
    const int level = hd[5];
    const uint64_t ne = le(hd + 6, 2);
    buf.resize(ne * (kKey + 8) + kKey);
    if (!pread_all(fd, buf.data(), buf.size(), fc.ub + a + 24)) return false;
    for (uint64_t i = 0; i < ne; ++i) {
      const uint8_t* k = &buf[i * (kKey + 8)];
      const uint64_t child = le(k + kKey, 8);
      if (level > 0) {
        stack.push_back(child);
        continue;
      }
      const uint64_t r0 = le(k + 8, 8), c0 = le(k + 16, 8);
      if (r0 % c[0] || c0 % c[1] || r0 / c[0] >= gr || c0 / c[1] >= gc) return false;
      const hsize_t g = (r0 / c[0]) * gc + c0 / c[1];
      if (have[g]) return false;
      have[g] = 1;
      ++got;
      tmh5_chunk& e = fc.ch[g];
      e.src_len = (int64_t)le(k, 4);
      e.raw_len = raw;
      e.row0 = (int32_t)r0;
      e.col0 = (int32_t)c0;
      e.flags = (le(k + 4, 4) & 1u) ? 1 : 0;
      e.reserved = 0;
      fc.addr[g] = (int64_t)(fc.ub + child);
    }
  }
  if (got != fc.n) return false;
  fc.bytes = 0;
  for (auto& e : fc.ch) {  // grid order, as chunks_by_hdf5
    e.src_off = fc.bytes;
    fc.bytes += e.src_len;
  }
  fc.parsed = true;
  return true;
}

}  // namespace

int tmh5_read_raw_chunks(const char* const* paths, int64_t n_files, int n_threads, uint8_t* blob,
                         int64_t blob_cap, tmh5_chunk* table, int64_t table_cap,
                         int64_t* blob_used, int64_t* n_chunks, int32_t* geom) {
  return guard([&] {
    silence();
    if (n_files < 0 || (n_files > 0 && !paths) || !blob_used || !n_chunks || !geom)
      throw H5Err{-22, "bad arguments"};
    *blob_used = 0;
    *n_chunks = 0;
    if (n_files == 0) return;
    int h = 0, w = 0, bits = 0;
    int rc = tmh5_channel_image_shape(paths[0], &h, &w, &bits);
    if (rc) throw H5Err{rc, g_err};
    const int esize = bits / 8;
    hsize_t ch[2] = {0, 0};
    std::vector<FileChunks> fc((size_t)n_files);
    for (int64_t i = 0; i < n_files; ++i) file_header(paths[i], i, h, w, esize, ch, fc[i]);
    const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(n_threads > 0 ? n_threads : 1, n_files));
    // the chunk indexes, in parallel outside the HDF5 lock; TMH5_CHUNK_INDEX:
    // "hdf5" = libhdf5's lookups only, "parse" = the parse only (tests)
    const char* ci = getenv("TMH5_CHUNK_INDEX");
    const bool use_hdf5 = ci && strcmp(ci, "hdf5") == 0;
    const bool parse_only = ci && strcmp(ci, "parse") == 0;
    {
      std::atomic<int64_t> next{0};
      auto parse = [&] {
        for (;;) {
          const int64_t i = next.fetch_add(1);
          if (i >= n_files) return;
          if (!use_hdf5) parse_chunk_index(paths[i], esize, ch, fc[i]);
        }
      };
      std::vector<std::thread> pool;
      for (int t = 1; t < nt; ++t) pool.emplace_back(parse);
      parse();
      for (auto& t : pool) t.join();
    }
    for (int64_t i = 0; i < n_files; ++i) {
      if (fc[i].parsed) continue;
      if (parse_only) throw H5Err{-95, std::string(paths[i]) + ": chunk index not parsed"};
      chunks_by_hdf5(paths[i], esize, ch, fc[i]);
    }
    int64_t total = 0, nch = 0;
    for (auto& f : fc) {
      total += f.bytes;
      nch += (int64_t)f.ch.size();
    }
    geom[0] = h;
    geom[1] = w;
    geom[2] = esize;
    geom[3] = (int32_t)ch[0];
    geom[4] = (int32_t)ch[1];
    *blob_used = total;
    *n_chunks = nch;
    if (total > blob_cap || nch > table_cap || (total && !blob) || (nch && !table))
      throw H5Err{-28, "raw chunk buffers too small"};
    // table: blob offsets and raw offsets (chunk raw bytes, file order)
    int64_t off = 0, k = 0;
    const int64_t raw = (int64_t)(ch[0] * ch[1]) * esize;
    for (auto& f : fc) {
      for (auto& e : f.ch) {
        tmh5_chunk t = e;
        t.src_off += off;
        t.raw_off = k * raw;
        table[k++] = t;
      }
      off += f.bytes;
    }
    // the bytes, one file per task, outside the HDF5 lock
    std::vector<int64_t> base((size_t)n_files, 0);
    for (int64_t i = 1; i < n_files; ++i) base[i] = base[i - 1] + fc[i - 1].bytes;
    std::atomic<int64_t> next{0};
    std::atomic<bool> failed{false};
    std::string first_err;
    std::mutex m;
    auto work = [&] {
      for (;;) {
        const int64_t i = next.fetch_add(1);
        if (i >= n_files || failed.load()) return;
        const int fd = open(paths[i], O_RDONLY);
        bool ok = fd >= 0;
        for (size_t j = 0; ok && j < fc[i].ch.size(); ++j) {
          uint8_t* dst = blob + base[i] + fc[i].ch[j].src_off;
          int64_t left = fc[i].ch[j].src_len, pos = fc[i].addr[j];
          while (left > 0) {
            const ssize_t r = pread(fd, dst, (size_t)left, (off_t)pos);
            if (r <= 0) {
              ok = false;
              break;
            }
            dst += r;
            pos += r;
            left -= r;
          }
        }
        if (fd >= 0) close(fd);
        if (!ok) {
          std::lock_guard<std::mutex> lk(m);
          if (!failed.exchange(true)) first_err = std::string(paths[i]) + ": reading chunks failed";
        }
      }
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < nt; ++t) pool.emplace_back(work);
    work();
    for (auto& t : pool) t.join();
    if (failed) throw H5Err{-5, first_err};
  });
}

int tmh5_read_channel_images(const char* const* paths, int64_t n_files, void* out, int n_threads) {
  return guard([&] {
    silence();
    if (n_files < 0 || ((!paths || !out) && n_files > 0)) throw H5Err{-22, "bad arguments"};
    if (n_files == 0) return;
    int h = 0, w = 0, bits = 0;
    int rc = tmh5_channel_image_shape(paths[0], &h, &w, &bits);
    if (rc) throw H5Err{rc, g_err};
    const int esize = bits / 8;
    const size_t img = (size_t)h * w * esize;
    const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(n_threads > 0 ? n_threads : 1, n_files));
    std::atomic<int64_t> next{0};
    std::atomic<bool> failed{false};
    std::string first_err;
    int first_code = 0;
    std::mutex m;
    auto work = [&] {
      for (;;) {
        const int64_t i = next.fetch_add(1);
        if (i >= n_files || failed.load()) return;
        try {
          read_one_parallel(paths[i], static_cast<uint8_t*>(out) + (size_t)i * img, h, w, esize);
        } catch (const H5Err& e) {
          std::lock_guard<std::mutex> lk(m);
          if (!failed.exchange(true)) {
            first_err = e.msg;
            first_code = e.code;
          }
        } catch (...) {
          std::lock_guard<std::mutex> lk(m);
          if (!failed.exchange(true)) {
            first_err = std::string(paths[i]) + ": read failed";
            first_code = -5;
          }
        }
      }
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < nt; ++t) pool.emplace_back(work);
    work();
    for (auto& t : pool) t.join();
    if (failed) throw H5Err{first_code, first_err};
  });
}

}  // extern "C"
