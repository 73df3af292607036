/*
 * pqgen.h — deterministic synthetic Parquet generator.
 *
 * Produces byte-identical files on any host: splitmix64 PRNG, doubles built
 * from integer bits (no libm).  Two page layouts:
 *   PQGEN_REF_LAYOUT    the reference writer's format (parquet_writer.cpp:
 *                       56-98 page split, 272 dictionary threshold,
 *                       rle_bp_encoder.hpp single-group bit-packed runs,
 *                       103-135 RLE-only levels).  Without footer padding the
 *                       bytes equal the reference ParquetWriter's output.
 *   PQGEN_ARROW_LAYOUT  fixed rows per page (default 20,000), hybrid runs with
 *                       bit-packed runs of up to 63 groups, RLE for runs >= 8.
 */
#ifndef PQGEN_H
#define PQGEN_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    PQGEN_DICT_STRINGS = 0, /* C2/C5: dictionary of random lowercase strings, runs of an index */
    PQGEN_COMMENT = 1,      /* C3: words from a fixed 36-word vocabulary, truncated            */
    PQGEN_UNIFORM = 2,      /* uniform random bits of the physical type                       */
    PQGEN_DOUBLE_RANGE = 3, /* C4 c3-c5: (u>>11)*2^-53*2000-1000                               */
    PQGEN_SMALL_INT = 4     /* uniform in [0, dict_size): low-cardinality fixed width          */
};
enum { PQGEN_REF_LAYOUT = 0, PQGEN_ARROW_LAYOUT = 1 };

typedef struct {
    const char* name;
    int32_t kind;       /* PQGEN_* kind                                          */
    int32_t type;       /* ParquetType (BOOLEAN..BYTE_ARRAY)                     */
    int32_t optional;   /* 1 = OPTIONAL (max_def 1), 0 = REQUIRED                */
    double null_frac;   /* iid NULL probability per row (OPTIONAL only)          */
    int32_t dict_size;  /* PQGEN_DICT_STRINGS / PQGEN_SMALL_INT cardinality      */
    int32_t len_min;    /* string length range [len_min, len_max)                */
    int32_t len_max;
    int32_t max_run;    /* PQGEN_DICT_STRINGS runs are 1 + U[0, max_run) rows    */
    int32_t force_plain;/* arrow layout: 1 = never dictionary-encode             */
} pqgen_col;

typedef struct {
    int32_t layout;         /* PQGEN_REF_LAYOUT / PQGEN_ARROW_LAYOUT                 */
    int32_t rows_per_page;  /* arrow layout rows per data page (0 -> 20000)          */
    int32_t footer_pad;     /* add a created_by string so the footer is >= 300 B     */
    int32_t first_rg;       /* generate row groups [first_rg, first_rg + nrg) of the */
                            /* logical file (each rank of a sharded run its own)     */
} pqgen_opts;

/* Build a whole file in memory.  *out is malloc'd; free with pqgen_free. */
int pqgen_build(const pqgen_col* cols, int ncols, int64_t rows_per_rg, int nrg, uint64_t seed,
                const pqgen_opts* opts, uint8_t** out, size_t* out_len);
void pqgen_free(void* p);

/* Per-column canonical dump (SURVEY §8 format) of the generated values of
 * row group `rg` — what a correct decoder must return. */
int pqgen_values_dump(const pqgen_col* col, int col_idx, int64_t rows, int rg, uint64_t seed,
                      uint8_t** out, size_t* out_len);

#ifdef __cplusplus
}
#endif
#endif
