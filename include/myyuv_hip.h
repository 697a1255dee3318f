/*
 * myyuv_hip.h — C ABI of the MI355X (gfx950) DCT codec: the drop-in boundary
 * for the reference's DCT compress/decompress path.
 *
 * The reference binds this path in two places (paths relative to
 * /root/reference/myyuv_lib/):
 *   - myyuv_yuv.hpp:111,116 / myyuv_yuv.cpp:130-160: YUV::compress_map[DCT][IYUV]
 *     and YUV::decompress_map[DCT][IYUV] (std::function plugin table), and
 *   - myyuv_DCT/DCT.hpp:16,25 (extern-declared at myyuv_yuv.cpp:9-14):
 *     myyuvDCT::compress_DCT_planar / decompress_DCT_planar.
 * Each entry point below says which of those it replaces.  The C++ adapter
 * that re-registers the maps through this ABI is
 * yuv-manipulations-2_amd/csrc/host/myyuv_yuv.cpp.
 *
 * Byte format: the payload handled here is exactly the DCTYUV stream the
 * reference writes after the 64-byte YUVHeader and the 3 quality bytes
 * (DCT.cpp:112-197, Huffman.cpp:279-326): u32 plane_size[3],
 * then per plane u32 nblocks, u32 content_size, u8 chunk_size[nblocks],
 * u8 content[content_size].  Frames are IYUV (4:2:0 planar, Y then U then V).
 *
 * Plain pointers and sizes only; no torch or HIP types in the signatures
 * (streams are passed as void* = hipStream_t).  All functions return 0 or a
 * MYYUV_E_* code; myyuv_hip_strerror() gives the reference's message for it.
 */
#ifndef MYYUV_HIP_H
#define MYYUV_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Error codes.  The string for each (myyuv_hip_strerror) is the exact
 * std::runtime_error text the reference throws at the cited line. */
#define MYYUV_OK 0
#define MYYUV_E_ARG 1             /* null pointer / bad handle (no reference counterpart) */
#define MYYUV_E_QUALITY 2         /* DCT.cpp:380,440 "Level of quality must be between 1 and 100" */
#define MYYUV_E_WIDTH 3           /* DCT.cpp:281,339 "Error. width % 8 must be 0" */
#define MYYUV_E_HEIGHT 4          /* DCT.cpp:284,342 "Error. height % 8 must be 0" */
#define MYYUV_E_CAPACITY 5        /* output buffer smaller than the payload (no reference counterpart) */
#define MYYUV_E_DCTYUV_SIZE 6     /* DCT.cpp:133,144 "DCTYUV load bad size" */
#define MYYUV_E_PLANE_SIZE 7      /* DCT.cpp:42,54 "DCTYUVPlane load bad size" */
#define MYYUV_E_PLANE_NBLK 8      /* DCT.cpp:48 "DCTYUVPlane load chunks_sizes_size bad size" */
#define MYYUV_E_PLANE_CONTENT 9   /* DCT.cpp:51 "DCTYUVPlane load content_size bad size" */
#define MYYUV_E_BAD_CODE 10       /* Huffman.cpp:121,130 "Huffman bad code" */
#define MYYUV_E_UNKNOWN_SYMBOL 11 /* Huffman.cpp:139 "Huffman unknown symbol" */
#define MYYUV_E_BAD_CHUNK 12      /* malformed chunk header/table (reference: assert / UB) */
#define MYYUV_E_HIP 13            /* HIP runtime failure */
#define MYYUV_E_NO_DEVICE 14      /* no gfx950 device / HIP unavailable */
#define MYYUV_E_BMP_INVALID 15    /* myyuv_yuv.cpp:514 "BMP is invalid" (width % 4, bit_count 0) */
#define MYYUV_E_BMP_SIGN 16       /* myyuv_bmp.cpp:98 "Unaccounted width and height sign" */
#define MYYUV_E_BMP_UNSUPPORTED 17 /* odd height or not 24/32 bpp (reference: assert, myyuv_yuv.cpp:92,97) */

typedef struct myyuv_hip_ctx* myyuv_hip_handle;

/* Context: one per (host thread, device).  Owns a HIP stream and the per-call
 * workspace (grown on demand, never freed inside a call); the host-buffer
 * entry points copy straight from / into the caller's pageable buffers.
 * Reentrant across contexts, as the
 * reference is (SURVEY.md §8b "Threading").  Calls through ONE context share
 * its workspace, so they run in call order even on different streams: a call
 * on a stream other than the previous call's makes its stream wait for the
 * previous call's work (an event recorded at the end of every call).  For
 * concurrency, use one context per stream. */
int myyuv_hip_create(int device, myyuv_hip_handle* out);
void myyuv_hip_destroy(myyuv_hip_handle h);
const char* myyuv_hip_strerror(int code);

/* Upper bound of the DCTYUV payload for a WxH IYUV frame (worst-case 160 B per
 * 8x8 block + headers); size the compress output buffer with it. */
uint32_t myyuv_dct_payload_bound(uint32_t width, uint32_t height);

/* Host-buffer compress: replaces myyuvDCT::compress_DCT_planar's data path
 * (DCT.cpp:371-430), i.e. what YUV::compress_map[DCT][IYUV] runs
 * (myyuv_yuv.cpp:132-142).  iyuv = W*H*3/2 bytes (Y, U, V planes as in
 * YUV::getYUVPlanes, myyuv_yuv.cpp:383-423).  Writes the DCTYUV payload to
 * `payload` (capacity `cap`) and its size to *payload_size.  The caller (C++
 * adapter) writes the 64-B header and the 3 quality bytes. */
int myyuv_gpu_dct_compress(myyuv_hip_handle h, const uint8_t* iyuv, uint32_t width,
                           uint32_t height, const uint8_t quality[3], uint8_t* payload,
                           uint32_t cap, uint32_t* payload_size);

/* Host-buffer decompress: replaces myyuvDCT::decompress_DCT_planar's data path
 * (DCT.cpp:432-488), what YUV::decompress_map[DCT][IYUV] runs
 * (myyuv_yuv.cpp:148-158).  Writes W*H*3/2 bytes to `iyuv`.  On a decode error
 * returns its code; *bad_block (optional) receives the global block index
 * (plane-major, row-major blocks) of the first failing block, -1 for header
 * errors. */
int myyuv_gpu_dct_decompress(myyuv_hip_handle h, const uint8_t* payload, uint32_t size,
                             uint32_t width, uint32_t height, const uint8_t quality[3],
                             uint8_t* iyuv, int64_t* bad_block);

/* Device-resident variants (HBM in, HBM out), asynchronous on `stream`
 * (hipStream_t; NULL = the context's stream).  Used by the batch driver and
 * the benchmark: no host synchronisation, no allocation once the workspace
 * has grown to the frame size (call myyuv_hip_reserve first to pre-size it).
 *   compress:   d_iyuv (W*H*3/2 B) -> d_payload (cap B), *d_payload_size (u32, device)
 *   decompress: d_payload + *d_payload_size (device u32) -> d_iyuv
 * Errors found on the device are collected in the context and returned by
 * myyuv_hip_sync_status. */
int myyuv_hip_reserve(myyuv_hip_handle h, uint32_t width, uint32_t height);
int myyuv_gpu_dct_compress_device(myyuv_hip_handle h, const void* d_iyuv, uint32_t width,
                                  uint32_t height, const uint8_t quality[3], void* d_payload,
                                  uint32_t cap, uint32_t* d_payload_size, void* stream);
int myyuv_gpu_dct_decompress_device(myyuv_hip_handle h, const void* d_payload,
                                    const uint32_t* d_payload_size, uint32_t cap, uint32_t width,
                                    uint32_t height, const uint8_t quality[3], void* d_iyuv,
                                    void* stream);
/* Batches: `nframes` frames of one geometry per launch of each kernel (the
 * batch configuration of SURVEY.md §8d; fills the GPU where one 4K frame
 * cannot).  Frame f at d_iyuv + f*W*H*3/2; payload f at d_payload + f*cap
 * (cap a multiple of 4 when nframes > 1), its size at d_payload_sizes[f].
 * A device-side error reports the batch-global block index
 * (f * blocks_per_frame + block) of the first failing block; a header error
 * of frame f > 0 reports f * blocks_per_frame.  Each frame's bytes are those
 * of the single-frame call.
 * Workspace (myyuv_hip_reserve_batch reserves it up front; the calls grow it
 * on demand): about 471 B per 8x8 block of the batch — the encoder's stage
 * (160 B: a tile's chunks, kMaxChunk per block, rounded up to whole 4-tile
 * K2 windows) and overflow slots (160 B per block: any block may exceed 8
 * distinct symbols, as nearly all of a noise frame's do, so the slots cannot
 * be sized from a typical list), the coefficients (128 B), the chunk offsets
 * (u32 srcoff, 4 B), the decoder's group offsets (4 B), the overflow worklist
 * (8 B: the CAP-16 tier's list and its rest list), the sizes and row masks
 * (2 B), K1's per-block words for K2 (4 B) and its exact-path list (0.25 B).
 * A 4032x3008 frame (284,256 blocks) takes ~134 MB: the bench's 24-frame
 * launch groups ~3.2 GB per context, its 4 contexts ~12.8 GB; a 16-frame
 * 8192x8192 batch ~11.9 GB (of 288 GB). */
int myyuv_hip_reserve_batch(myyuv_hip_handle h, uint32_t width, uint32_t height, uint32_t nframes);
int myyuv_gpu_dct_compress_batch_device(myyuv_hip_handle h, const void* d_iyuv, uint32_t nframes,
                                        uint32_t width, uint32_t height, const uint8_t quality[3],
                                        void* d_payload, uint32_t cap, uint32_t* d_payload_sizes,
                                        void* stream);
int myyuv_gpu_dct_decompress_batch_device(myyuv_hip_handle h, const void* d_payload,
                                          const uint32_t* d_payload_sizes, uint32_t cap,
                                          uint32_t nframes, uint32_t width, uint32_t height,
                                          const uint8_t quality[3], void* d_iyuv, void* stream);
/* BMP -> IYUV: replaces YUV(const BMP&, IYUV), i.e.
 * YUV::bmp_to_yuv_map[IYUV] (myyuv_yuv.cpp:88-128) over BMP::colorData
 * (myyuv_bmp.cpp:77-101).  `bmp_data` is BMP::data — the pixel array as stored
 * in the file (BGR or BGRA, bit_count 24 or 32, |width| % 4 == 0 so rows are
 * unpadded); `width` / `height` are the header's signed fields, whose signs
 * select colorData's orientation (height > 0: bottom-up rows; width < 0:
 * pixel order reversed).  Writes |width|*|height|*3/2 IYUV bytes.  The C++
 * adapter checks the rest of BMP::isValidHeader and writes the YUV header. */
int myyuv_gpu_bmp_to_iyuv(myyuv_hip_handle h, const uint8_t* bmp_data, int32_t width,
                          int32_t height, uint16_t bit_count, uint8_t* iyuv);
/* Device-resident variant, asynchronous on `stream` (NULL = the context's);
 * argument errors are returned at once. */
int myyuv_gpu_bmp_to_iyuv_device(myyuv_hip_handle h, const void* d_bmp_data, int32_t width,
                                 int32_t height, uint16_t bit_count, void* d_iyuv, void* stream);

/* Host-buffer batches (many frames per call; §7 step 9:
 * transfers overlapped with the kernels).  The batch runs in chunks of up to
 * 8 frames through two device slots: chunk k's host -> device copies, chunk
 * k-1's kernels (one launch per kernel for the chunk) and chunk k-2's
 * device -> host copies run at once, on three streams.  Every frame's bytes
 * are those of the single-frame calls; the calls return when every output
 * is in host memory.  Replaces a loop of YUV::compress / YUV::decompress
 * (myyuv_cli/main.cpp:151-207) over many frames.
 *
 * Compress: frames[f] -> payload f, written to the buffer alloc(user, f,
 * size) returns once the frame's size is known (NULL: MYYUV_E_CAPACITY and
 * the call stops); sizes[f] = its size.  alloc runs on the calling thread,
 * in frame order. */
typedef uint8_t* (*myyuv_payload_alloc_fn)(void* user, uint32_t frame, uint32_t size);
int myyuv_gpu_dct_compress_frames(myyuv_hip_handle h, const uint8_t* const* frames, uint32_t nframes,
                                  uint32_t width, uint32_t height, const uint8_t quality[3],
                                  myyuv_payload_alloc_fn alloc, void* user, uint32_t* sizes);
/* Contiguous form: frame f at iyuv + f*W*H*3/2 -> payload f at payloads +
 * f*cap.  MYYUV_E_CAPACITY when a payload exceeds `cap` (sizes[] hold the
 * sizes up to that frame). */
int myyuv_gpu_dct_compress_batch(myyuv_hip_handle h, const uint8_t* iyuv, uint32_t nframes,
                                 uint32_t width, uint32_t height, const uint8_t quality[3],
                                 uint8_t* payloads, uint32_t cap, uint32_t* sizes);
/* Decompress: stream f (payloads[f], sizes[f] bytes) -> frames[f]
 * (W*H*3/2 bytes).  Every stream's header is checked first (the
 * single-frame call's DCTYUV::load checks); a decode error stops the call
 * with *bad_block the batch-global index of the failing block (frame f's
 * block g: f * blocks-per-frame + g). */
int myyuv_gpu_dct_decompress_frames(myyuv_hip_handle h, const uint8_t* const* payloads, const uint32_t* sizes,
                                    uint32_t nframes, uint32_t width, uint32_t height, const uint8_t quality[3],
                                    uint8_t* const* frames, int64_t* bad_block);
/* Contiguous form: stream f at payloads + f*cap -> frame f at iyuv + f*W*H*3/2. */
int myyuv_gpu_dct_decompress_batch(myyuv_hip_handle h, const uint8_t* payloads, const uint32_t* sizes,
                                   uint32_t cap, uint32_t nframes, uint32_t width, uint32_t height,
                                   const uint8_t quality[3], uint8_t* iyuv, int64_t* bad_block);

/* Waits for `stream`, returns (and clears) the first device-side error since
 * the last call; *bad_block as above. */
int myyuv_hip_sync_status(myyuv_hip_handle h, void* stream, int64_t* bad_block);

/* Per-kernel timing (HIP events around each launch, on the launch stream).
 * enable=1 starts recording; myyuv_hip_kernel_stats fills, per kernel id
 * (MYYUV_K_*), the summed milliseconds and launch count since enabling.
 * Times are kernel execution times (start/stop stamped from the dispatch
 * packet, as rocprofv3's kernel trace). */
#define MYYUV_K_FDCT 0       /* K1 fdct_quant */
#define MYYUV_K_HUFF_ENC 1   /* K2 huff_encode (CAP=8 pass over every block) */
#define MYYUV_K_SCAN 2       /* single-pass chunk-size scan (both directions; decode: + header checks) */
#define MYYUV_K_COMPACT 3    /* K4 stream writer: look-back scan + tiles into the DCTYUV stream */
#define MYYUV_K_ENCODE_TILE 4 /* fused single-pass encoder K1 + K2 (MYYUV_ENCODER=fused) */
#define MYYUV_K_HUFF_DEC 5   /* K5 huff_decode */
#define MYYUV_K_IDCT 6       /* K6 dequant_idct */
#define MYYUV_K_HUFF_WIDE 7  /* K2 overflow pass, lane per block (long worklists) */
#define MYYUV_K_HUFF_R16 8   /* K2 overflow tier 1: register-resident, up to 16 symbols, lane per block */
#define MYYUV_K_HUFF_WAVE 9  /* K2 overflow pass, wave per block (short worklists) */
#define MYYUV_K_BMP 10       /* K7 bmp_to_iyuv (BMP -> IYUV conversion) */
#define MYYUV_K_FDCT_FIX 11  /* K1's exact path for the units K1 listed (fdct_fix) */
#define MYYUV_K_COUNT 12
int myyuv_hip_profile(myyuv_hip_handle h, int enable);
/* As myyuv_hip_profile, but stamps only the kernels whose bit (1 << MYYUV_K_*)
 * is set in `mask` (0 disables): event stamping costs host and queue time per
 * launch, so a timed region profiles just the kernel it reports on. */
int myyuv_hip_profile_kernels(myyuv_hip_handle h, uint32_t mask);
int myyuv_hip_kernel_stats(myyuv_hip_handle h, double ms[MYYUV_K_COUNT],
                           int64_t launches[MYYUV_K_COUNT]);

/* Block-level entry points for known-answer tests (device round trip of one
 * batch of blocks).  coef is zig-zag ordered int16[64] per block; the encoder
 * rejects (MYYUV_E_ARG) coefficients outside [-1024, 1023], the 11-bit range
 * the chunk format carries and K1 produces (DCT.cpp:276). */
int myyuv_gpu_fdct_blocks(myyuv_hip_handle h, const uint8_t* px, uint32_t nblocks,
                          const float qtable[64], int16_t* coef_zz);
int myyuv_gpu_huff_encode_blocks(myyuv_hip_handle h, const int16_t* coef_zz, uint32_t nblocks,
                                 uint8_t* chunks160, uint8_t* sizes);

#ifdef __cplusplus
}
#endif
#endif /* MYYUV_HIP_H */
