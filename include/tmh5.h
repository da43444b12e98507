/*
 * tmh5.h — C-ABI of libtmh5.so: the illumination path's HDF5 files, read and
 * written through libhdf5 (1.10, /opt/conda) instead of h5py.
 *
 * Replaces, with the on-disk layout unchanged:
 *   tmlib/models/file.py:440-456  IllumstatsFile.put  (DatasetWriter.write x4,
 *                                 tmlib/writers.py:322-389)
 *   tmlib/models/file.py:420-438  IllumstatsFile.get  (DatasetReader.read,
 *                                 tmlib/readers.py:367-389)
 *   tmlib/models/file.py:353-363  ChannelImageFile.put (gzip /array)
 *   tmlib/models/file.py:322-351  ChannelImageFile.get
 * Return 0 on success, negative errno-style code on failure
 * (-2: dataset missing -> KeyError, -22: bad argument, -5: HDF5 error).
 */
#ifndef TMH5_H
#define TMH5_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

const char* tmh5_last_error(void);

int tmh5_write_illumstats(const char* path, int height, int width, const double* mean,
                          const double* std_, int64_t n_quantiles, const double* keys,
                          const int64_t* values);
int tmh5_illumstats_shape(const char* path, int* height, int* width, int64_t* n_quantiles);
/* any output may be NULL (that dataset is skipped) */
int tmh5_read_illumstats(const char* path, double* mean, double* std_, double* keys,
                         int64_t* values);

/* bits: 8 or 16; gzip_level < 0 writes an uncompressed contiguous dataset */
int tmh5_write_channel_image(const char* path, int height, int width, int bits, const void* data,
                             int gzip_level);
/* same with explicit chunk extents (0: the default whole-row ~256 KiB chunks),
 * e.g. to reproduce h5py's automatic 2-D chunking of the reference's files */
int tmh5_write_channel_image_chunked(const char* path, int height, int width, int bits,
                                     const void* data, int gzip_level, int chunk_rows,
                                     int chunk_cols);
int tmh5_channel_image_shape(const char* path, int* height, int* width, int* bits);
int tmh5_read_channel_image(const char* path, void* out);
/* n_files channel images (same shape and dtype) into out[n][H][W], decoded by
 * n_threads workers: raw deflate chunks from HDF5, zlib inflate in parallel
 * (the input path of run_job / configs[4]). */
int tmh5_read_channel_images(const char* const* paths, int64_t n_files, void* out, int n_threads);

/* The still-compressed chunks of n_files channel images for the GPU inflate
 * (libtmhip tmh_inflate_device / tmh_place_chunks_device; tmh5_chunk has the
 * layout of tmh_zchunk): every chunk's zlib stream is copied into blob
 * (blob_cap bytes) and described by one table entry (table_cap entries) --
 * src_off / src_len in blob, raw_off / raw_len of its decompressed bytes in a
 * raw buffer of *n_chunks full chunks (file order), image = the file's index,
 * (row0, col0) its origin, flags 1 = stored (the filter was skipped).
 * geom = {height, width, elem_bytes, chunk_rows, chunk_cols}.  *blob_used and
 * *n_chunks are set also when a capacity is too small (-28, nothing read).
 * Files must share shape, dtype and chunk shape and be chunked with exactly
 * the deflate filter, all chunks written (-95 otherwise: read those with
 * tmh5_read_channel_images).  The HDF5 metadata is read under libhdf5's
 * lock, the chunk bytes with pread() by n_threads workers outside it. */
typedef struct tmh5_chunk {
  int64_t src_off, src_len, raw_off, raw_len, image;
  int32_t row0, col0, flags, reserved;
} tmh5_chunk;
int tmh5_read_raw_chunks(const char* const* paths, int64_t n_files, int n_threads, uint8_t* blob,
                         int64_t blob_cap, tmh5_chunk* table, int64_t table_cap,
                         int64_t* blob_used, int64_t* n_chunks, int32_t* geom);

#ifdef __cplusplus
}
#endif
#endif /* TMH5_H */
