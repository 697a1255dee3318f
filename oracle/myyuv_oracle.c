/*
 * myyuv_oracle.c — CPU restatement of the reference DCT codec path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (libmyyuv_hip.so, the
 * C++ host library, the CLI) links, loads or calls this file.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it, and only
 * as the checker / CPU baseline.
 *
 * Parity status: PINNED.  This restatement reproduces the reference's golden
 * files byte-for-byte (images/chef-with-trumpet-DCT-50.myyuv, -DCT-90.myyuv
 * from chef-with-trumpet.myyuv; decode of chef-with-trumpet-big-DCT-50.myyuv
 * re-encodes to the same bytes) and is cross-checked against the reference
 * sources compiled into oracle/_ref/ (see oracle/Makefile, tests/test_oracle.py).
 *
 * Written from the byte-format description, citing the
 * reference function each piece restates.  Paths are relative to
 * /root/reference/myyuv_lib/.
 *
 * Build: gcc -O2 -ffp-contract=off -fopenmp (never -march=native: FMA
 * contraction changes the coefficients).
 */
#include <math.h>
#include <stdint.h>
#include <limits.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "myyuv_oracle.h"

/* ---------------------------------------------------------------------------
 * Constant tables: myyuv_DCT/DCT.cpp:199-230 (JPEG Annex K.1 / K.2 and the
 * float-literal DCT-II basis; literal values, not cos(), they are asymmetric).
 * ------------------------------------------------------------------------- */
static const float k_lum_q[64] = {
    16, 11, 10, 16, 24,  40,  51,  61,  12, 12, 14, 19, 26,  58,  60,  55,
    14, 13, 16, 24, 40,  57,  69,  56,  14, 17, 22, 29, 51,  87,  80,  62,
    18, 22, 37, 56, 68,  109, 103, 77,  24, 35, 55, 64, 81,  104, 113, 92,
    49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99};

static const float k_chroma_q[64] = {
    17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99,
    24, 26, 56, 99, 99, 99, 99, 99, 47, 66, 99, 99, 99, 99, 99, 99,
    99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99,
    99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99};

static const float k_dct[64] = {
    0.3535533845424652f,  0.3535533845424652f,  0.3535533845424652f,  0.3535533845424652f,
    0.3535533845424652f,  0.3535533845424652f,  0.3535533845424652f,  0.3535533845424652f,
    0.4903925955295563f,  0.4157347679138184f,  0.277785062789917f,   0.09754510968923569f,
    -0.09754515439271927f, -0.2777851521968842f, -0.4157347977161407f, -0.4903926253318787f,
    0.4619397222995758f,  0.1913416981697083f,  -0.1913417428731918f, -0.4619397819042206f,
    -0.4619397222995758f, -0.1913415491580963f, 0.1913417875766754f,  0.4619397521018982f,
    0.4157347679138184f,  -0.09754515439271927f, -0.4903926253318787f, -0.2777849733829498f,
    0.2777851819992065f,  0.4903925955295563f,  0.09754502773284912f, -0.4157348573207855f,
    0.3535533547401428f,  -0.3535533547401428f, -0.353553295135498f,  0.3535534739494324f,
    0.3535533547401428f,  -0.3535535931587219f, -0.3535532355308533f, 0.3535533845424652f,
    0.277785062789917f,   -0.4903926253318787f, 0.09754519909620285f, 0.4157346487045288f,
    -0.4157348573207855f, -0.09754510223865509f, 0.4903926253318787f,  -0.2777853906154633f,
    0.1913416981697083f,  -0.4619397222995758f, 0.4619397521018982f,  -0.1913419365882874f,
    -0.1913414746522903f, 0.4619396328926086f,  -0.4619398415088654f, 0.1913419365882874f,
    0.09754510968923569f, -0.2777849733829498f, 0.4157346487045288f,  -0.4903925657272339f,
    0.4903926849365234f,  -0.4157347679138184f, 0.2777855396270752f,  -0.09754576534032822f};

/* Huffman.cpp:32-34 */
static const uint8_t k_zigzag[64] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
    41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
    30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

const uint8_t* oracle_zigzag(void) { return k_zigzag; }
const float* oracle_dct_matrix(void) { return k_dct; }

/* DCT.cpp:286-290 (and the identical loop at :344-348). */
void oracle_qtable(int q, int chroma, float out[64]) {
    const float* base = chroma ? k_chroma_q : k_lum_q;
    const float fq = (float)q;
    const float mul = (fq >= 50.5f) ? (100.0f - fq) / 50.0f : 50.0f / fq;
    for (int i = 0; i < 64; i++) {
        float v = roundf(base[i] * mul);
        if (v < 1.0f) v = 1.0f;
        if (v > 255.0f) v = 255.0f;
        out[i] = v;
    }
}

/* Forward transform of one block: DCT.cpp:232-254 (squareMatrixMul, MulT),
 * :269-277 (applyDCTBlock), :301-305 (gather, -128).  Every sum starts from
 * 0.0f and adds fp32-rounded products in ascending k (no FMA). */
void oracle_fdct_block(const uint8_t px[64], const float Q[64], int16_t coef[64]) {
    float x[64], t[64];
    for (int i = 0; i < 64; i++) x[i] = (float)px[i] - 128.0f;
    for (int i = 0; i < 8; i++)
        for (int j = 0; j < 8; j++) {
            float s = 0.0f;
            for (int k = 0; k < 8; k++) {
                float p = k_dct[i * 8 + k] * x[k * 8 + j];
                s = s + p;
            }
            t[i * 8 + j] = s;
        }
    for (int i = 0; i < 8; i++)
        for (int j = 0; j < 8; j++) {
            float s = 0.0f;
            for (int k = 0; k < 8; k++) {
                float p = t[i * 8 + k] * k_dct[j * 8 + k];
                s = s + p;
            }
            coef[i * 8 + j] = (int16_t)roundf(s / Q[i * 8 + j]);
        }
}

/* Inverse transform of one block: DCT.cpp:256-266 (squareMatrixMulT2, Mul),
 * :325-335 (restoreDCTBlock), :358-362 (round, +128, clamp). */
void oracle_idct_block(const int16_t coef[64], const float Q[64], uint8_t px[64]) {
    float z[64], u[64];
    for (int i = 0; i < 64; i++) z[i] = (float)coef[i] * Q[i];
    for (int i = 0; i < 8; i++)
        for (int j = 0; j < 8; j++) {
            float s = 0.0f;
            for (int k = 0; k < 8; k++) {
                float p = k_dct[k * 8 + i] * z[k * 8 + j];
                s = s + p;
            }
            u[i * 8 + j] = s;
        }
    for (int i = 0; i < 8; i++)
        for (int j = 0; j < 8; j++) {
            float s = 0.0f;
            for (int k = 0; k < 8; k++) {
                float p = u[i * 8 + k] * k_dct[k * 8 + j];
                s = s + p;
            }
            int v = (int)roundf(s) + 128;
            px[i * 8 + j] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
        }
}

/* ---------------------------------------------------------------------------
 * libstdc++ std::unordered_map<int16_t,uint8_t> iteration-order model.
 * Restates the behaviour Huffman.cpp:173-197 depends on:
 * singly linked node list + per-bucket "before" pointers, prime rehash policy
 * (13 -> 29 -> 59 -> 127 buckets for <= 65 elements), bucket-front insertion,
 * re-insertion walk on rehash; hash(int16 v) = (size_t)(int64)v.
 * ------------------------------------------------------------------------- */
#define HM_NIL 0xFF
#define HM_HEAD 0xFE /* "before" pointer == the list head sentinel */

typedef struct {
    int16_t key[66];
    uint8_t cnt[66];
    uint8_t nxt[66];
    uint8_t live[66];
    uint8_t bucket_before[128];
    uint8_t head; /* first node, HM_NIL if empty */
    uint32_t nb;  /* bucket count */
    uint32_t next_resize;
    uint32_t n;     /* live elements */
    uint32_t nodes; /* allocated nodes */
} hashorder_t;

static uint32_t hm_bucket(int16_t v, uint32_t nb) {
    uint64_t h = (uint64_t)(int64_t)v;
    return (uint32_t)(h % nb);
}

static void hm_init(hashorder_t* m) {
    m->head = HM_NIL;
    m->nb = 1;
    m->next_resize = 0;
    m->n = 0;
    m->nodes = 0;
    for (int i = 0; i < 128; i++) m->bucket_before[i] = HM_NIL;
}

/* _Prime_rehash_policy::_M_next_bkt restricted to the sizes reachable here. */
static uint32_t hm_next_bkt(uint32_t x, uint32_t* next_resize) {
    static const uint8_t fast[14] = {2, 2, 2, 3, 5, 5, 7, 7, 11, 11, 11, 11, 13, 13};
    static const uint32_t primes[] = {17, 19, 23, 29, 31, 37, 41, 43, 47, 53, 59, 61, 67, 71,
                                      73, 79, 83, 89, 97, 103, 109, 113, 127, 131, 137, 139, 149,
                                      151, 157, 163, 167, 173, 179, 181, 191, 193, 197, 199, 211,
                                      223, 227, 229, 233, 239, 241, 251, 257};
    if (x < 14) {
        uint32_t r = x == 0 ? 1 : fast[x];
        *next_resize = r;
        return r;
    }
    for (size_t i = 0; i < sizeof(primes) / sizeof(primes[0]); i++)
        if (primes[i] >= x) {
            *next_resize = primes[i];
            return primes[i];
        }
    abort();
}

static uint8_t* hm_link(hashorder_t* m, uint8_t before) {
    return before == HM_HEAD ? &m->head : &m->nxt[before];
}

/* _M_insert_bucket_begin */
static void hm_insert_bucket_begin(hashorder_t* m, uint32_t bkt, uint8_t node) {
    if (m->bucket_before[bkt] != HM_NIL) {
        uint8_t* l = hm_link(m, m->bucket_before[bkt]);
        m->nxt[node] = *l;
        *l = node;
    } else {
        m->nxt[node] = m->head;
        m->head = node;
        if (m->nxt[node] != HM_NIL) m->bucket_before[hm_bucket(m->key[m->nxt[node]], m->nb)] = node;
        m->bucket_before[bkt] = HM_HEAD;
    }
}

/* _M_rehash_aux(n, true_type) */
static void hm_rehash(hashorder_t* m, uint32_t nb) {
    uint8_t p = m->head;
    m->head = HM_NIL;
    for (int i = 0; i < 128; i++) m->bucket_before[i] = HM_NIL;
    uint32_t bbegin = 0;
    while (p != HM_NIL) {
        uint8_t next = m->nxt[p];
        uint32_t b = hm_bucket(m->key[p], nb);
        if (m->bucket_before[b] == HM_NIL) {
            m->nxt[p] = m->head;
            m->head = p;
            m->bucket_before[b] = HM_HEAD;
            if (m->nxt[p] != HM_NIL) m->bucket_before[bbegin] = p;
            bbegin = b;
        } else {
            uint8_t* l = hm_link(m, m->bucket_before[b]);
            m->nxt[p] = *l;
            *l = p;
        }
        p = next;
    }
    m->nb = nb;
}

static int hm_find(const hashorder_t* m, int16_t v) {
    uint32_t b = hm_bucket(v, m->nb);
    if (m->bucket_before[b] == HM_NIL) return -1;
    uint8_t p = m->bucket_before[b] == HM_HEAD ? m->head : m->nxt[m->bucket_before[b]];
    while (p != HM_NIL && hm_bucket(m->key[p], m->nb) == b) {
        if (m->key[p] == v) return p;
        p = m->nxt[p];
    }
    return -1;
}

/* operator[]: find or insert with value 0; returns node index. */
static int hm_subscript(hashorder_t* m, int16_t v) {
    int f = hm_find(m, v);
    if (f >= 0) return f;
    /* _M_need_rehash(bkt_count, element_count, 1) */
    if (m->n + 1 > m->next_resize) {
        uint32_t minb = m->n + 1;
        if (m->next_resize == 0 && minb < 11) minb = 11;
        if (minb >= m->nb) {
            uint32_t want = minb + 1;
            if (want < 2 * m->nb) want = 2 * m->nb;
            uint32_t nb = hm_next_bkt(want, &m->next_resize);
            hm_rehash(m, nb);
        } else {
            m->next_resize = m->nb;
        }
    }
    uint8_t node = (uint8_t)m->nodes++;
    m->key[node] = v;
    m->cnt[node] = 0;
    m->live[node] = 1;
    hm_insert_bucket_begin(m, hm_bucket(v, m->nb), node);
    m->n++;
    return node;
}

/* erase(key): unlink, no rehash, others keep their order. */
static void hm_erase(hashorder_t* m, int node) {
    uint32_t b = hm_bucket(m->key[node], m->nb);
    uint8_t before = m->bucket_before[b];
    uint8_t* l = hm_link(m, before);
    while (*l != node) l = &m->nxt[*l];
    uint8_t next = m->nxt[node];
    uint8_t prev_link_owner = (l == &m->head) ? HM_HEAD : (uint8_t)(l - m->nxt);
    int is_first = (prev_link_owner == before);
    if (is_first) {
        /* _M_remove_bucket_begin */
        if (next == HM_NIL || hm_bucket(m->key[next], m->nb) != b) {
            if (next != HM_NIL) m->bucket_before[hm_bucket(m->key[next], m->nb)] = before;
            m->bucket_before[b] = HM_NIL;
        }
    } else if (next != HM_NIL) {
        uint32_t nbk = hm_bucket(m->key[next], m->nb);
        if (nbk != b) m->bucket_before[nbk] = prev_link_owner;
    }
    *l = next;
    m->live[node] = 0;
    m->n--;
}

/* ---------------------------------------------------------------------------
 * std::priority_queue<node, vector, Compare{a.freq > b.freq}> — libstdc++
 * push_heap / pop_heap (__adjust_heap + __push_heap) restated on arrays.
 * Huffman.cpp:204-217, Huffman.hpp:36-40.
 * ------------------------------------------------------------------------- */
typedef struct {
    uint8_t id[128];
    uint8_t freq[128];
    int len;
} heap_t;

static void heap_sift_up(heap_t* h, int hole, int top, uint8_t id, uint8_t fr) {
    int parent = (hole - 1) / 2;
    while (hole > top && h->freq[parent] > fr) {
        h->id[hole] = h->id[parent];
        h->freq[hole] = h->freq[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    h->id[hole] = id;
    h->freq[hole] = fr;
}

static void heap_push(heap_t* h, uint8_t id, uint8_t fr) {
    h->len++;
    heap_sift_up(h, h->len - 1, 0, id, fr);
}

static void heap_pop(heap_t* h, uint8_t* id, uint8_t* fr) {
    *id = h->id[0];
    *fr = h->freq[0];
    int len = h->len - 1;
    if (len > 0) {
        uint8_t vid = h->id[len], vfr = h->freq[len];
        h->id[len] = h->id[0];
        h->freq[len] = h->freq[0];
        /* __adjust_heap(first, 0, len, value) */
        int hole = 0, child = 0;
        while (child < (len - 1) / 2) {
            child = 2 * (child + 1);
            if (h->freq[child] > h->freq[child - 1]) child--;
            h->id[hole] = h->id[child];
            h->freq[hole] = h->freq[child];
            hole = child;
        }
        if ((len & 1) == 0 && child == (len - 2) / 2) {
            child = 2 * (child + 1);
            h->id[hole] = h->id[child - 1];
            h->freq[hole] = h->freq[child - 1];
            hole = child - 1;
        }
        heap_sift_up(h, hole, 0, vid, vfr);
    }
    h->len = len;
}

/* ---------------------------------------------------------------------------
 * Per-block entropy coder: Huffman::fromData (Huffman.cpp:172-241) +
 * generateCodeLength (:71-83) + generateCanonicalTree (:86-103) +
 * Huffman::dump / pack11bit (:279-326, :36-52).
 * Returns the chunk size (7..155) written to chunk[].
 * ------------------------------------------------------------------------- */
int oracle_huff_encode_block(const int16_t coef[64], uint8_t* chunk) {
    int16_t zd[64];
    int trail = 0;
    for (int i = 0; i < 64; i++) {
        zd[i] = coef[k_zigzag[i]];
        trail = (zd[i] == 0) ? trail + 1 : 0;
    }
    int msz = 64 - trail;

    hashorder_t m;
    hm_init(&m);
    for (int i = 0; i < 64; i++) m.cnt[hm_subscript(&m, zd[i])]++;
    int z = hm_find(&m, 0);
    if (z >= 0) m.cnt[z] -= (uint8_t)trail;
    z = hm_subscript(&m, 0); /* freq[0] == 0 probe (inserts) */
    if (m.cnt[z] == 0) {
        if (msz == 0) {
            m.cnt[z] = 1;
            msz = 1;
        } else {
            hm_erase(&m, z);
        }
    }

    /* leaves in iteration order -> heap */
    int nleaf = 0;
    int16_t leaf_key[64];
    uint8_t leaf_len[64];
    heap_t h;
    h.len = 0;
    for (uint8_t p = m.head; p != HM_NIL; p = m.nxt[p]) {
        leaf_key[nleaf] = m.key[p];
        heap_push(&h, (uint8_t)nleaf, m.cnt[p]);
        nleaf++;
    }
    /* merges: internal nodes get ids 64.. */
    uint8_t parent[128];
    int nint = 0;
    while (h.len > 1) {
        uint8_t li, lf, ri, rf;
        heap_pop(&h, &li, &lf);
        heap_pop(&h, &ri, &rf);
        uint8_t id = (uint8_t)(64 + nint++);
        parent[li] = id;
        parent[ri] = id;
        heap_push(&h, id, (uint8_t)(lf + rf));
    }
    if (nint == 0) {
        leaf_len[0] = 1; /* single leaf: depth 0 -> length 1 */
    } else {
        uint8_t depth[128];
        depth[64 + nint - 1] = 0;
        for (int k = nint - 2; k >= 0; k--) depth[64 + k] = depth[parent[64 + k]] + 1;
        for (int j = 0; j < nleaf; j++) leaf_len[j] = depth[parent[j]] + 1;
    }

    /* canonical order: by length, then by symbol value */
    int16_t sym[64];
    uint8_t slen[64];
    int ns = 0;
    for (int L = 1; L <= 8; L++) {
        int start = ns;
        for (int j = 0; j < nleaf; j++)
            if (leaf_len[j] == L) {
                int16_t v = leaf_key[j];
                int pos = ns++;
                while (pos > start && sym[pos - 1] > v) {
                    sym[pos] = sym[pos - 1];
                    slen[pos] = slen[pos - 1];
                    pos--;
                }
                sym[pos] = v;
                slen[pos] = (uint8_t)L;
            }
    }
    /* canonical codes */
    uint8_t code[64];
    {
        unsigned c = 0, prev = 0;
        for (int i = 0; i < ns; i++) {
            c <<= (slen[i] - prev);
            prev = slen[i];
            code[i] = (uint8_t)c;
            c++;
        }
    }

    /* serialise */
    int pos = 3;
    int i = 0;
    while (i < ns) {
        int L = slen[i];
        int j = i;
        while (j < ns && slen[j] == L) j++;
        int cnt = j - i;
        while (cnt > 0) {
            int g = cnt > 32 ? 32 : cnt;
            chunk[pos++] = (uint8_t)(((L - 1) << 5) | (g - 1));
            int nbytes = (g * 11 + 7) / 8;
            memset(chunk + pos, 0, (size_t)nbytes);
            for (int t = 0; t < g; t++) {
                int16_t v = sym[i + t];
                unsigned u = v < 0 ? (unsigned)(2048 + v) : (unsigned)v;
                unsigned bit = (unsigned)t * 11u;
                for (int b = 0; b < 11; b++)
                    if (u & (1u << b)) chunk[pos + (bit + b) / 8] |= (uint8_t)(1u << ((bit + b) % 8));
            }
            pos += nbytes;
            i += g;
            cnt -= g;
        }
    }
    int table_bytes = pos - 3;
    int nbits = 0;
    int data_start = pos;
    for (int s = 0; s < msz; s++) {
        int idx = -1;
        for (int t = 0; t < ns; t++)
            if (sym[t] == zd[s]) {
                idx = t;
                break;
            }
        int L = slen[idx];
        for (int b = 0; b < L; b++) {
            int bitv = (code[idx] >> (L - 1 - b)) & 1;
            int at = nbits + b;
            if ((at & 7) == 0) chunk[data_start + at / 8] = 0;
            if (bitv) chunk[data_start + at / 8] |= (uint8_t)(1u << (at & 7));
        }
        nbits += L;
    }
    int enc_bytes = (nbits + 7) / 8;
    chunk[0] = (uint8_t)(nbits & 0xFF);
    chunk[1] = (uint8_t)(nbits >> 8);
    chunk[2] = (uint8_t)table_bytes;
    return 3 + table_bytes + enc_bytes;
}

/* ---------------------------------------------------------------------------
 * Huffman::fromDump + unpack11bit + decodeSymbol + decodeFromTreeData
 * (Huffman.cpp:243-277, :54-69, :106-154).  Output: 64 int16 in natural
 * (row-major) order.  Returns 0 or an ORACLE_E_* code.  uint8 arithmetic of
 * decodeSymbol is kept (code/first wrap) so corrupt chunks fail the same way.
 * ------------------------------------------------------------------------- */
int oracle_huff_decode_block(const uint8_t* chunk, int size, int16_t coef[64]) {
    memset(coef, 0, 64 * sizeof(int16_t));
    if (size < 3) return ORACLE_E_BAD_CHUNK;
    unsigned nbits = (unsigned)chunk[0] | ((unsigned)chunk[1] << 8);
    unsigned tbytes = chunk[2];
    unsigned enc_bytes = (nbits + 7) / 8;
    if (nbits > 512 || 3 + tbytes + enc_bytes > (unsigned)size) return ORACLE_E_BAD_CHUNK;
    int16_t sym[8][64];
    int cnt[9] = {0};
    unsigned i = 3;
    while (i - 3 < tbytes) {
        uint8_t info = chunk[i++];
        int L = (info >> 5) + 1;
        int c = (info & 31) + 1;
        unsigned nbytes = ((unsigned)c * 11 + 7) / 8;
        if (i + nbytes > 3 + tbytes || cnt[L] + c > 64) return ORACLE_E_BAD_CHUNK;
        for (int t = 0; t < c; t++) {
            unsigned bit = (unsigned)t * 11u, u = 0;
            for (int b = 0; b < 11; b++)
                if (chunk[i + (bit + b) / 8] & (1u << ((bit + b) % 8))) u |= 1u << b;
            sym[L - 1][cnt[L]++] = (int16_t)(u >= 1024 ? (int)u - 2048 : (int)u);
        }
        i += nbytes;
    }
    if (i - 3 != tbytes) return ORACLE_E_BAD_CHUNK;
    const uint8_t* bits = chunk + 3 + tbytes;
    unsigned bp = 0;
    int j = 0;
    while (bp < nbits && j < 64) {
        uint8_t code = 0, first = 0;
        int found = 0;
        int16_t v = 0;
        for (int L = 1; L <= 8; L++) {
            if (bp >= nbits) return ORACLE_E_BAD_CODE;
            code |= (uint8_t)((bits[bp >> 3] >> (bp & 7)) & 1);
            bp++;
            if ((int)code < cnt[L] + (int)first) {
                if (cnt[L] == 0) return ORACLE_E_BAD_CODE;
                v = sym[L - 1][(uint8_t)(code - first)];
                found = 1;
                break;
            }
            first = (uint8_t)(first + cnt[L]);
            first = (uint8_t)(first << 1);
            code = (uint8_t)(code << 1);
        }
        if (!found) return ORACLE_E_UNKNOWN_SYMBOL;
        coef[k_zigzag[j++]] = v;
    }
    return 0;
}

/* ---------------------------------------------------------------------------
 * Plane and frame level: applyDCTPlane / restoreDCTPlane (DCT.cpp:279-365),
 * compress_DCT_planar / decompress_DCT_planar (:371-488), DCTYUV(Plane)
 * load/dump (:16-197).  OpenMP mirrors the reference's block loop
 * (schedule(dynamic,1) over blocks, nested over planes).
 * ------------------------------------------------------------------------- */
static void plane_dims(uint32_t w, uint32_t h, int p, uint32_t* pw, uint32_t* ph) {
    *pw = p == 0 ? w : w / 2;
    *ph = p == 0 ? h : h / 2;
}

static size_t plane_offset(uint32_t w, uint32_t h, int p) {
    return p == 0 ? 0 : (p == 1 ? (size_t)w * h : (size_t)w * h * 5 / 4);
}

/* applyDCTPlane / restoreDCTPlane dimension checks (DCT.cpp:280-285,
 * :338-343), evaluated plane by plane in serial order. */
static int check_dims(uint32_t w, uint32_t h) {
    for (int p = 0; p < 3; p++) {
        uint32_t pw, ph;
        plane_dims(w, h, p, &pw, &ph);
        if (pw % 8 != 0) return ORACLE_E_WIDTH;
        if (ph % 8 != 0) return ORACLE_E_HEIGHT;
    }
    return 0;
}

uint32_t oracle_payload_bound(uint32_t w, uint32_t h) {
    uint64_t nb = (uint64_t)w * h / 64 + 2 * ((uint64_t)w * h / 256);
    return (uint32_t)(12 + 3 * 8 + nb + nb * ORACLE_MAX_CHUNK);
}

int oracle_compress(const uint8_t* iyuv, uint32_t w, uint32_t h, const uint8_t q[3],
                    uint8_t* payload, uint32_t cap, uint32_t* out_size) {
    for (int p = 0; p < 3; p++)
        if (q[p] < 1 || q[p] > 100) return ORACLE_E_QUALITY;
    int e = check_dims(w, h);
    if (e) return e;
    uint32_t off = 12;
    uint32_t plane_sizes[3];
    for (int p = 0; p < 3; p++) {
        uint32_t pw, ph;
        plane_dims(w, h, p, &pw, &ph);
        const uint8_t* src = iyuv + plane_offset(w, h, p);
        float Q[64];
        oracle_qtable(q[p], p != 0, Q);
        uint32_t bw = pw / 8, bh = ph / 8, nblk = bw * bh;
        uint8_t* chunks = (uint8_t*)malloc((size_t)nblk * ORACLE_MAX_CHUNK);
        uint8_t* sizes = (uint8_t*)malloc(nblk);
#pragma omp parallel for schedule(dynamic, 1)
        for (int64_t k = 0; k < (int64_t)nblk; k++) {
            uint32_t by = (uint32_t)k / bw, bx = (uint32_t)k % bw;
            uint8_t px[64];
            int16_t c[64];
            for (int r = 0; r < 8; r++)
                memcpy(px + r * 8, src + (size_t)(by * 8 + r) * pw + bx * 8, 8);
            oracle_fdct_block(px, Q, c);
            sizes[k] = (uint8_t)oracle_huff_encode_block(c, chunks + (size_t)k * ORACLE_MAX_CHUNK);
        }
        uint64_t content = 0;
        for (uint32_t k = 0; k < nblk; k++) content += sizes[k];
        uint64_t need = (uint64_t)off + 8 + nblk + content;
        if (need > cap) {
            free(chunks);
            free(sizes);
            return ORACLE_E_CAPACITY;
        }
        uint32_t c32 = (uint32_t)content;
        memcpy(payload + off, &nblk, 4);
        memcpy(payload + off + 4, &c32, 4);
        memcpy(payload + off + 8, sizes, nblk);
        uint8_t* dst = payload + off + 8 + nblk;
        for (uint32_t k = 0; k < nblk; k++) {
            memcpy(dst, chunks + (size_t)k * ORACLE_MAX_CHUNK, sizes[k]);
            dst += sizes[k];
        }
        plane_sizes[p] = 8 + nblk + c32;
        off += plane_sizes[p];
        free(chunks);
        free(sizes);
    }
    memcpy(payload, plane_sizes, 12);
    *out_size = off;
    return 0;
}

/* DCTYUV::load + DCTYUVPlane::load size checks (DCT.cpp:39-62, :130-159),
 * then per plane the dims check and the block loop.  Stricter than the
 * reference where it is undefined: a zero plane size, fewer chunk sizes than
 * blocks, or chunk sizes summing past content_size are errors here. */
int oracle_decompress(const uint8_t* payload, uint32_t size, uint32_t w, uint32_t h,
                      const uint8_t q[3], uint8_t* iyuv) {
    for (int p = 0; p < 3; p++)
        if (q[p] < 1 || q[p] > 100) return ORACLE_E_QUALITY;
    if (size <= 12) return ORACLE_E_DCTYUV_SIZE;
    uint32_t ps[3];
    memcpy(ps, payload, 12);
    uint64_t total = 12 + (uint64_t)ps[0] + ps[1] + ps[2];
    if (total > size) return ORACLE_E_DCTYUV_SIZE;
    uint64_t poff[3];
    poff[0] = 12;
    poff[1] = poff[0] + ps[0];
    poff[2] = poff[1] + ps[1];
    uint32_t hn[3], hc[3];
    for (int p = 0; p < 3; p++) {
        if (ps[p] <= 8) return ORACLE_E_PLANE_SIZE;
        memcpy(&hn[p], payload + poff[p], 4);
        memcpy(&hc[p], payload + poff[p] + 4, 4);
        if (hn[p] == 0) return ORACLE_E_PLANE_NBLK;
        if (hc[p] == 0) return ORACLE_E_PLANE_CONTENT;
        if (8 + (uint64_t)hn[p] + hc[p] > ps[p]) return ORACLE_E_PLANE_SIZE;
    }
    int err = 0;
    for (int p = 0; p < 3 && !err; p++) {
        uint32_t pw, ph;
        plane_dims(w, h, p, &pw, &ph);
        if (pw % 8 != 0) return ORACLE_E_WIDTH;
        if (ph % 8 != 0) return ORACLE_E_HEIGHT;
        uint32_t bw = pw / 8, bh = ph / 8, nblk = bw * bh;
        if (hn[p] < nblk) return ORACLE_E_PLANE_NBLK;
        const uint8_t* sizes = payload + poff[p] + 8;
        const uint8_t* content = sizes + hn[p];
        uint32_t* pos = (uint32_t*)malloc((size_t)nblk * 4);
        uint64_t acc = 0;
        for (uint32_t k = 0; k < nblk; k++) {
            pos[k] = (uint32_t)acc;
            acc += sizes[k];
        }
        if (acc > hc[p]) {
            free(pos);
            return ORACLE_E_PLANE_CONTENT;
        }
        float Q[64];
        oracle_qtable(q[p], p != 0, Q);
        uint8_t* dst = iyuv + plane_offset(w, h, p);
        int64_t bad_blk = INT64_MAX;
        int bad_err = 0;
#pragma omp parallel for schedule(dynamic, 1)
        for (int64_t k = 0; k < (int64_t)nblk; k++) {
            uint32_t by = (uint32_t)k / bw, bx = (uint32_t)k % bw;
            int16_t c[64];
            uint8_t px[64];
            int e = oracle_huff_decode_block(content + pos[k], sizes[k], c);
            if (e) {
#pragma omp critical
                if (k < bad_blk) {
                    bad_blk = k;
                    bad_err = e;
                }
            }
            oracle_idct_block(c, Q, px);
            for (int r = 0; r < 8; r++) memcpy(dst + (size_t)(by * 8 + r) * pw + bx * 8, px + r * 8, 8);
        }
        free(pos);
        err = bad_err;
    }
    return err;
}

int oracle_num_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

void oracle_set_num_threads(int n) {
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
#else
    (void)n;
#endif
}

/* ------------------------------------------------------------------------
 * BMP -> IYUV: YUV(const BMP&, IYUV), i.e.
 * bmp_to_yuv_map[IYUV] (myyuv_yuv.cpp:88-128) over BMP::colorData
 * (myyuv_bmp.cpp:77-101), with getYUV444FromRGB2x2 (myyuv_yuv.cpp:34-52) and
 * divide_roundnearest<uint8_t> (:20-27).
 *
 * bmp_data is BMP::data (the pixel array as stored in the file: BGR(A),
 * `bit_count` bits per pixel, no row padding since width % 4 == 0).
 * colorData's orientation: width > 0, height < 0 -> as stored; width < 0,
 * height > 0 -> pixel order reversed; both > 0 -> rows bottom-up.
 * Numerics as the reference's x86-64 -O3 build: fp32 products and sums left
 * to right, no contraction; float -> uint8_t casts truncate toward zero
 * through a 32-bit integer and keep the low byte (cvttss2si); the 4-term
 * chroma sum wraps mod 256 (a saturated-blue quad has Cb 0).
 * ---------------------------------------------------------------------- */
static uint8_t bmp_cast_u8(float x) { return (uint8_t)(int32_t)x; }

static void bmp_yuv444(const uint8_t* px, uint8_t* y, uint8_t* cb, uint8_t* cr) {
  const float B = (float)px[0], G = (float)px[1], R = (float)px[2];
  const float Y = 0.299f * R + 0.587f * G + 0.114f * B;
  *y = bmp_cast_u8(Y);
  *cb = (uint8_t)(bmp_cast_u8((B - Y) * 0.564f) + 128);
  *cr = (uint8_t)(bmp_cast_u8((R - Y) * 0.713f) + 128);
}

int oracle_bmp_to_iyuv(const uint8_t* bmp_data, int32_t width, int32_t height, uint32_t bit_count,
                       uint8_t* iyuv) {
  const uint32_t W = (uint32_t)(width < 0 ? -(int64_t)width : width);
  const uint32_t H = (uint32_t)(height < 0 ? -(int64_t)height : height);
  if (W % 4 != 0 || bit_count == 0) return ORACLE_E_BMP_INVALID;
  if (!((width > 0 && height < 0) || (width < 0 && height > 0) || (width > 0 && height > 0)))
    return ORACLE_E_BMP_SIGN;
  if ((bit_count != 24 && bit_count != 32) || H % 2 != 0) return ORACLE_E_BMP_UNSUPPORTED;
  const uint32_t bpp = bit_count / 8;
  const size_t npx = (size_t)W * H;
  uint8_t* u = iyuv + npx;
  uint8_t* v = iyuv + npx + npx / 4;
  for (uint32_t j = 0; j < H; j += 2)
    for (uint32_t i = 0; i < W; i += 2) {
      uint8_t y4[4], cb4[4], cr4[4];
      for (int q = 0; q < 4; q++) {
        const uint32_t r = j + (q >> 1), c = i + (q & 1);
        size_t src;
        if (width > 0 && height < 0)
          src = (size_t)r * W + c;
        else if (width < 0)
          src = npx - 1 - ((size_t)r * W + c);
        else
          src = (size_t)(H - 1 - r) * W + c;
        bmp_yuv444(bmp_data + src * bpp, &y4[q], &cb4[q], &cr4[q]);
        iyuv[(size_t)r * W + c] = y4[q];
      }
      uint8_t scb = 0, scr = 0;
      for (int q = 0; q < 4; q++) {
        scb = (uint8_t)(scb + (uint8_t)((cb4[q] + 2) / 4));
        scr = (uint8_t)(scr + (uint8_t)((cr4[q] + 2) / 4));
      }
      const size_t k = (size_t)(j / 2) * (W / 2) + i / 2;
      u[k] = scb;
      v[k] = scr;
    }
  return 0;
}
