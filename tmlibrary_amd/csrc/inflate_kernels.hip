// GPU inflate of HDF5 gzip chunks (gfx950 / MI355X) -- the site-image input
// path of the corilla job.
//
// Reference: tmlib/models/file.py:322-351 (ChannelImageFile.get) and
// tmlib/readers.py:367-389 (DatasetReader.read): h5py reads the gzip-filtered
// /array dataset, i.e. libhdf5's deflate filter runs zlib's inflate on every
// chunk (files written by tmlib/models/file.py:353-363 / writers.py:384-387).
// Each HDF5 chunk is an independent zlib stream (RFC 1950 header, RFC 1951
// deflate blocks, Adler-32 trailer), so a batch of sites is thousands of
// independent streams: here one LANE decodes one stream, 64 streams per
// wave, and the GPU's thousands of waves hide the serial decode's latency.
// Host cores then only move compressed bytes (raw chunks read straight from
// the files, libtmh5) and the PCIe link carries compressed data.
//
// Per lane (LDS, interleaved [index][lane] so the 64 lanes' table reads fall
// in different banks): the literal/length and distance codes as canonical
// Huffman tables -- left-justified limit per code length, symbol base per
// length, symbols in code order -- decoded by a 4-step binary search over the
// 15 code lengths on the bit-reversed 15-bit peek; the dynamic block header's
// code lengths; a count/offset scratch for the table build.  The lane's loop
// is a flat state machine (one deflate symbol, or one whole block header, per
// iteration) so lanes at different points of their streams stay converged
// on the symbol path.  Output bytes go to the chunk's region of a raw
// buffer; back-references read the lane's own earlier output (same thread,
// same address: program order).  Adler-32 is checked like zlib's inflate.
// tmh_place_chunks_device then moves each chunk's rows into [image][H][W]
// (edge chunks carry padding past the dataset extent).
#include "common.h"
#include "inflate_core.h"

namespace tmh {

__global__ __launch_bounds__(kZW) void k_inflate(const uint8_t* __restrict__ src, int64_t src_bytes,
                                                 const tmh_zchunk* __restrict__ chunks,
                                                 int64_t n_chunks, uint8_t* __restrict__ dst,
                                                 int64_t dst_bytes, int32_t* __restrict__ status) {
  __shared__ ZShared z;
  const int lane = threadIdx.x;
  const int64_t ci = (int64_t)blockIdx.x * kZW + lane;
  if (ci >= n_chunks) return;
  status[ci] = inflate_stream(src, src_bytes, chunks[ci], dst, dst_bytes, z, lane);
}

// Chunk i's raw bytes (chunk_rows x chunk_cols elements, row-major) into
// image c.image of [*][height][width] at (row0, col0), clipped to the
// dataset's extent.  One workgroup per (chunk, 64 rows), 16-byte copies
// where the row segments allow, else per element.
__global__ __launch_bounds__(256) void k_place_chunks(const uint8_t* __restrict__ raw,
                                                      const tmh_zchunk* __restrict__ chunks,
                                                      int64_t n_chunks, int height, int width,
                                                      int esize, int chunk_rows, int chunk_cols,
                                                      uint8_t* __restrict__ images) {
  const int64_t ci = blockIdx.x;
  if (ci >= n_chunks) return;
  const tmh_zchunk c = chunks[ci];
  const int rows = min(chunk_rows, height - c.row0);
  const int cols = min(chunk_cols, width - c.col0);
  if (rows <= 0 || cols <= 0) return;
  const int64_t rb = (int64_t)cols * esize;                       // bytes per placed row
  const int64_t sstride = (int64_t)chunk_cols * esize;             // raw row stride
  const int64_t dstride = (int64_t)width * esize;
  const uint8_t* s = raw + c.raw_off;
  uint8_t* d = images + (c.image * height + c.row0) * dstride + (int64_t)c.col0 * esize;
  const bool v16 = ((reinterpret_cast<uintptr_t>(s) | reinterpret_cast<uintptr_t>(d)) & 15) == 0 &&
                   (rb & 15) == 0 && (sstride & 15) == 0 && (dstride & 15) == 0;
  for (int r = blockIdx.y; r < rows; r += gridDim.y) {
    const uint8_t* sr = s + r * sstride;
    uint8_t* dr = d + r * dstride;
    if (v16) {
      for (int64_t i = threadIdx.x; i < rb / 16; i += 256)
        reinterpret_cast<uint4*>(dr)[i] = reinterpret_cast<const uint4*>(sr)[i];
    } else {
      for (int64_t i = threadIdx.x; i < rb; i += 256) dr[i] = sr[i];
    }
  }
}

void launch_inflate(const uint8_t* src, int64_t src_bytes, const tmh_zchunk* chunks,
                    int64_t n_chunks, uint8_t* dst, int64_t dst_bytes, int32_t* status,
                    hipStream_t s) {
  if (n_chunks <= 0) return;
  ProfScope prof("inflate", s);
  hipLaunchKernelGGL(k_inflate, dim3((unsigned)cdiv(n_chunks, kZW)), dim3(kZW), 0, s, src,
                     src_bytes, chunks, n_chunks, dst, dst_bytes, status);
  TMH_HIP(hipGetLastError());
}

void launch_place_chunks(const uint8_t* raw, const tmh_zchunk* chunks, int64_t n_chunks,
                         int height, int width, int esize, int chunk_rows, int chunk_cols,
                         uint8_t* images, hipStream_t s) {
  if (n_chunks <= 0) return;
  ProfScope prof("place_chunks", s);
  const unsigned ry = (unsigned)std::min<int64_t>(64, std::max(1, chunk_rows));
  hipLaunchKernelGGL(k_place_chunks, dim3((unsigned)n_chunks, ry), dim3(256), 0, s, raw, chunks,
                     n_chunks, height, width, esize, chunk_rows, chunk_cols, images);
  TMH_HIP(hipGetLastError());
}

}  // namespace tmh
