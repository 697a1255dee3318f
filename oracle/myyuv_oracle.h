/*
 * myyuv_oracle.h — CPU restatement of the reference DCT codec (TEST
 * INFRASTRUCTURE ONLY; see myyuv_oracle.c header).  Error codes follow the
 * product's MYYUV_HIP_E_* numbering (include/myyuv_hip.h) so tests can compare
 * error behaviour directly.
 */
#ifndef MYYUV_ORACLE_H
#define MYYUV_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORACLE_MAX_CHUNK 160

#define ORACLE_E_QUALITY 2        /* "Level of quality must be between 1 and 100" */
#define ORACLE_E_WIDTH 3          /* "Error. width % 8 must be 0" */
#define ORACLE_E_HEIGHT 4         /* "Error. height % 8 must be 0" */
#define ORACLE_E_CAPACITY 5       /* output buffer too small */
#define ORACLE_E_DCTYUV_SIZE 6    /* "DCTYUV load bad size" */
#define ORACLE_E_PLANE_SIZE 7     /* "DCTYUVPlane load bad size" */
#define ORACLE_E_PLANE_NBLK 8     /* "DCTYUVPlane load chunks_sizes_size bad size" */
#define ORACLE_E_PLANE_CONTENT 9  /* "DCTYUVPlane load content_size bad size" */
#define ORACLE_E_BAD_CODE 10      /* "Huffman bad code" */
#define ORACLE_E_UNKNOWN_SYMBOL 11 /* "Huffman unknown symbol" */
#define ORACLE_E_BAD_CHUNK 12     /* malformed chunk (reference: UB / assert) */

#define ORACLE_E_BMP_INVALID 15    /* "BMP is invalid" */
#define ORACLE_E_BMP_SIGN 16       /* "Unaccounted width and height sign" */
#define ORACLE_E_BMP_UNSUPPORTED 17 /* odd dimensions / not 24 or 32 bpp (reference: assert) */

const uint8_t* oracle_zigzag(void);
const float* oracle_dct_matrix(void);
void oracle_qtable(int q, int chroma, float out[64]);
void oracle_fdct_block(const uint8_t px[64], const float Q[64], int16_t coef[64]);
void oracle_idct_block(const int16_t coef[64], const float Q[64], uint8_t px[64]);
int oracle_huff_encode_block(const int16_t coef[64], uint8_t* chunk);
int oracle_huff_decode_block(const uint8_t* chunk, int size, int16_t coef[64]);
uint32_t oracle_payload_bound(uint32_t w, uint32_t h);
int oracle_compress(const uint8_t* iyuv, uint32_t w, uint32_t h, const uint8_t q[3],
                    uint8_t* payload, uint32_t cap, uint32_t* out_size);
int oracle_decompress(const uint8_t* payload, uint32_t size, uint32_t w, uint32_t h,
                      const uint8_t q[3], uint8_t* iyuv);
int oracle_bmp_to_iyuv(const uint8_t* bmp_data, int32_t width, int32_t height, uint32_t bit_count,
                       uint8_t* iyuv);
int oracle_num_threads(void);
void oracle_set_num_threads(int n);

#ifdef __cplusplus
}
#endif
#endif
