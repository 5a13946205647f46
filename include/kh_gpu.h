/*
 * kh_gpu.h -- C ABI of the MI355X keyhunt engine (libkh_gpu.so).
 *
 * The reference (naanprofit/keyhunt) has no plugin API: its hot path is file-static C++ driven by
 * globals.  The seams this ABI replaces are the bodies of its worker threads:
 *
 *   kh_scan            <- thread_process, one N_SEQUENTIAL_MAX chunk      keyhunt.cpp:3265-3861
 *                         (group walk 3349-3461, hash160/xpoint probes 3475-3830, bloom_check +
 *                          searchbinary 3065-3089, parity fix-up 3619-3636)
 *   kh_set_targets     <- readFileAddress/forceReadFileAddress/...XPoint  keyhunt.cpp:7239-7490
 *                         + initBloomFilter 7605-7626 + _sort 1359-1364
 *   kh_bsgs_setup      <- BSGS parameter block                            keyhunt.cpp:1454-1842
 *   kh_bsgs_build      <- thread_bPload / thread_bPload_2blooms + bsgs_sort keyhunt.cpp:5284-5644, 2466-2503
 *   kh_bsgs_scan       <- thread_process_bsgs (sequential), bases of 2N   keyhunt.cpp:4549-4888
 *                         with bsgs_secondcheck (GPU) / bsgs_thirdcheck    keyhunt.cpp:5151-5248
 *
 * Conventions: plain C types only; 256-bit scalars and coordinates are 32-byte BIG-endian
 * (Int::Get32Bytes); every call returns 0 on success or a negative KH_E* code (never exits);
 * calls on one context are not re-entrant, contexts on different devices are independent;
 * the host owns every buffer passed in, the library owns device memory inside the context.
 * The engine never falls back to the CPU: if the HIP code object cannot run, calls fail.
 */
#ifndef KH_GPU_H
#define KH_GPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KH_ABI_VERSION 1

/* error codes */
#define KH_OK 0
#define KH_E_ARG -1        /* invalid argument */
#define KH_E_HIP -2        /* HIP runtime error (see kh_last_error) */
#define KH_E_NOMEM -3      /* device or host allocation failed */
#define KH_E_STATE -4      /* call out of order (e.g. scan before targets) */
#define KH_E_OVERFLOW -5   /* caller's output array too small (count is still reported) */
#define KH_E_BSGS_N -6     /* BSGS: n has no exact square root / sqrt(n) not a multiple of 1024 */
#define KH_E_RANGE -7      /* BSGS: range smaller than N ("[E] the given range is small") */
#define KH_E_IO -8         /* table file missing, short or not writable (see kh_last_error) */
#define KH_E_FORMAT -9     /* table file of another N/k, or its sha256 checksum does not match */

/* scan modes (-m) and search kinds (-l) */
#define KH_MODE_ADDRESS 0  /* -m address / -m rmd160: hash160 probes */
#define KH_MODE_XPOINT 1   /* -m xpoint: X[0..20) probes */
#define KH_MODE_ETH 2      /* -m address|rmd160 -c eth: Keccak-256(X||Y)[12..32) probes (the search kind is
                              ignored; keyhunt.cpp:3524-3548, 3703-3760, 5663-5669).  With KH_MODE_ENDO the
                              reference's six images: eth of P, -P, beta P, -beta P, beta P (again, its
                              slip at 3533) and -beta^2 P, each hit keyed as 3736-3744 derives it */
#define KH_MODE_ENDO 0x10  /* OR into the mode: -e, also probe (beta*X, Y) and (beta^2*X, Y), i.e. keys
                              lambda*k and lambda^2*k (keyhunt.cpp:3408-3440, 3476-3830) */
#define KH_SEARCH_COMPRESS 0
#define KH_SEARCH_UNCOMPRESS 1
#define KH_SEARCH_BOTH 2   /* reference default (FLAGSEARCH = 2) */

/* layer-1 (bloom_bP) layouts for kh_bsgs_set_layer1 */
#define KH_LAYER1_REFERENCE 0  /* the reference's bit layout (bloom/bloom.cpp): bit-identical tables */
#define KH_LAYER1_BLOCKED 1    /* default: split-block filter, an item's 16 bits in one 16-byte block chosen by
                                  the x-coordinate's own words (3x the bits per shard, FP 6.6e-7 vs 1e-6); one
                                  16-B load per probe.  Layers 2/3 stay in the reference layout, so refinement
                                  and found keys are unchanged */

/* hit kinds */
#define KH_KIND_02 0       /* hash160(02||X) matched */
#define KH_KIND_03 1       /* hash160(03||X) matched */
#define KH_KIND_04 2       /* hash160(04||X||Y) matched */
#define KH_KIND_XPOINT 3   /* X[0..20) matched */
#define KH_KIND_ETH 5      /* Ethereum address matched (key printed by writekeyeth) */
/* with KH_MODE_ENDO, kind also carries the image and (for 04 hashes) the Y sign: */
#define KH_KIND_ENDO1 0x10 /* matched on (beta*X, Y): key = lambda*k (+- as reported) */
#define KH_KIND_ENDO2 0x20 /* matched on (beta^2*X, Y): key = lambda^2*k */
#define KH_KIND_NEGY 0x40  /* 04||X||-Y (or, -c eth, -Y) matched: key negated */
/* -e -c eth: ETH | ENDO2 without NEGY is the reference's repeated beta P image (slot 4), reported
   after its ETH | ENDO1 twin with key n - lambda^2 k, as the reference prints it */

typedef struct kh_ctx kh_ctx;

/* one confirmed hit of kh_scan: the private key as the reference would print it */
typedef struct {
  uint8_t key[32];      /* big-endian; already negated (n - k) where the reference negates */
  uint64_t offset;      /* key offset from the chunk start (before negation) */
  uint32_t kind;        /* KH_KIND_* */
  uint32_t compressed;  /* 1 -> writekey(true, ...), 0 -> writekey(false, ...) */
} kh_hit;

/* BSGS parameters exactly as the reference derives them */
typedef struct {
  uint64_t n;           /* BSGS_N (rounded down to a multiple of M) */
  uint64_t m, m2, m3;   /* bsgs_m, bsgs_m2, bsgs_m3 */
  uint64_t aux;         /* bsgs_aux = N / M */
  uint64_t cycles;      /* ceil(aux / 1024) 1024-point groups per base */
  uint64_t bloom_bits[3], bloom_bytes[3];  /* per shard, layers 1..3 */
  uint32_t bloom_hashes[3];
  uint32_t layer1_layout; /* KH_LAYER1_*; for BLOCKED, bloom_bits[0] is the bit count rounded to whole blocks */
} kh_bsgs_info;

/* one key found by kh_bsgs_scan */
typedef struct {
  uint32_t target;      /* index into the targets given to kh_bsgs_set_targets */
  uint32_t pad;
  uint8_t key[32];      /* big-endian private key */
} kh_bsgs_found;

/* ---- context ------------------------------------------------------------------------------ */
int kh_device_count(int *count);
/* free and total device memory of `device` (hipMemGetInfo): hosts that stack several contexts on
 * one device check kh_bsgs_memory against it before building their tables */
int kh_device_memory(int device, uint64_t *free_bytes, uint64_t *total_bytes);
int kh_open(int device, kh_ctx **out);
int kh_close(kh_ctx *ctx);
const char *kh_strerror(int code);
const char *kh_last_error(kh_ctx *ctx);
int kh_abi_version(void);
/* lanes per walk launch (0 = automatic); groups (of 1024 points) per lane per launch (0 = auto) */
int kh_set_geometry(kh_ctx *ctx, uint32_t lanes, uint32_t groups_per_launch);
/* free the walks' device buffers (lane centres, scalars, inversion pad: up to 64 GB) between jobs;
 * the next scan allocates them again and starts its lanes afresh.  Tables and targets stay. */
int kh_release_walk(kh_ctx *ctx);
/* the BSGS walk's placement calibration (DESIGN.md §2 "Placement"): a context's first large calls walk
 * their parts on candidate placements of the inversion pad (a second pad of the same size, or 2^20
 * lanes when the device has no room for one), then of layer 1 (a copy), keeping the fastest of each.
 * *lanes = the lane count kept (0 = the pad stage not yet run), rates[0] = giant points/s of the pad
 * placement kept, rates[1] = of the best other one */
int kh_bsgs_geometry(kh_ctx *ctx, uint32_t *lanes, double rates[2]);
/* both stages of the placement calibration: rates[0..1] = the pad placement kept / the best other one,
 * rates[2..3] = the layer-1 placement kept / the other one (0 = stage not run).  Returns 1 when the
 * calibration is complete, 0 while stages remain. */
int kh_bsgs_placement(kh_ctx *ctx, double rates[4]);
/* diagnostics (DESIGN.md §2 "Placement"): where the BSGS walk's buffers sit in the device's virtual
 * address space.  out[0..1] = layer-1 address and bytes, out[2..3] = the inversion pad's, out[4..5] =
 * layer 2's, out[6] = lanes allocated, out[7] = pad rows per lane.  Engine-only: the reference has no
 * counterpart. */
int kh_debug_layout(kh_ctx *ctx, uint64_t out[8]);
/* diagnostics (DESIGN.md §2 "Placement"): give device buffers fresh allocations, taken while the old
 * ones are held, contents copied: which = 1 layer 1, 2 the inversion pad, 4 the lane centres and scalars,
 * 8 the walks' delta tables, 16 layers 2 and 3, 32 a new walk stream (bits may be combined).  Results
 * are unchanged. */
int kh_debug_replace(kh_ctx *ctx, uint32_t which);
/* diagnostics: enqueue about `ms` milliseconds of a VALU-dense load (no memory traffic) on the walk's
 * stream, left in flight (the board's clock/power operating point study, DESIGN.md §2 "Placement") */
int kh_debug_burn(kh_ctx *ctx, double ms);
int kh_synchronize(kh_ctx *ctx);

/* ---- address / rmd160 / xpoint ------------------------------------------------------------ */
/* rows: n x 20 bytes (hash160s, or X[0..20) for xpoint), any order.  bloom_items: the element
 * count the reference sizes its bloom with (numberItems), 0 -> n.  Sorts the table, builds the
 * reference-layout bloom (bloom_init2(max(10000, items), 1e-6)) and uploads both. */
int kh_set_targets(kh_ctx *ctx, const uint8_t *rows, uint64_t n, uint64_t bloom_items);
/* -m vanity targets instead (addvanity / processOneVanity, keyhunt.cpp:6739-6866, 6970-7035):
 * ranges = n x {A[20], B[20]} hash160 bounds (inclusive), probe_len = the prefix length the bloom
 * keys on (vanity_rmd_minimun_bytes_check_length, 1..20), bloom_items = the reference's item count
 * (vanity_rmd_total).  Following kh_scan calls in the hash160 modes report every point whose
 * hash lies in a range (vanityrmdmatch, 6677-6703), with the same key resolution as -m address.
 * kh_set_targets switches back to exact targets. */
int kh_set_vanity(kh_ctx *ctx, const uint8_t *ranges, uint64_t n, uint32_t probe_len, uint64_t bloom_items);
/* Scan keys start + i*stride, i in [0, n_keys) (n_keys a multiple of 1024; stride NULL -> 1).
 * Returns the confirmed hits in the order one reference thread prints them.  A call that starts
 * where the previous kh_scan of this context ended (same mode, stride and n_keys) reuses its
 * lanes instead of starting them again: sequential chunks are cheaper, results are the same. */
int kh_scan(kh_ctx *ctx, const uint8_t start[32], const uint8_t stride[32], uint64_t n_keys, uint32_t mode,
            uint32_t search, kh_hit *hits, uint32_t cap, uint32_t *n_hits);
/* The device bytes one context's kh_scan of n_keys-key chunks holds at the default geometry, exact
 * targets (the inversion pad -- 2^20 lanes x 4096-point groups for the 2^32-key chunks of -m xpoint and
 * -l compress, half of it for xpoint's sparse pad -- lane centres, comb, hit buffer; target tables come
 * on top).  Hosts that stack contexts on one device check it against kh_device_memory first.  With
 * --rmd-batch-size (kh_set_rmd_batch) a chunk needs less. */
int kh_scan_memory(uint64_t n_keys, uint32_t mode, uint32_t search, uint64_t *needed_bytes);
/* -m rmd160 --rmd-batch-size (keyhunt.cpp:815-829, 3301-3307): group = the reference's clamped
 * rmd_batch_size (a multiple of 4 in [4, 1024]; 1024 or 0 = the ordinary walk).  Below 1024 the
 * following hash160 kh_scan calls reproduce the reference's groups of `group` keys exactly as it
 * computes them: its batch inversion then runs over a partly zero IntGroup and returns 0 for every
 * inverse, so each group holds one real point (its centre, slot group/2) and group - 1 points
 * x = -(C.x + (i+1)D.x) that are no multiples of G; a chunk of n_keys becomes ceil(n_keys/group)
 * whole groups (it overshoots its end like the reference's do-while), and hits on those points
 * carry the key of their slot with the reference's key resolution.  KH_MODE_ADDRESS and
 * KH_MODE_ETH (-m rmd160 -c eth), exact targets. */
int kh_set_rmd_batch(kh_ctx *ctx, uint32_t group);

/* ---- BSGS --------------------------------------------------------------------------------- */
/* layer-1 layout for the next kh_bsgs_setup (KH_LAYER1_BLOCKED unless changed) */
int kh_bsgs_set_layer1(kh_ctx *ctx, uint32_t layout);
/* -z (FLAGBLOOMMULTIPLIER, keyhunt.cpp:1111-1117) for the next kh_bsgs_setup: initBloomFilter sizes a
 * shard of more than 10000 items for mult x items entries (keyhunt.cpp:7608), so the three layers'
 * geometry -- and their -S files -- follow it as the reference's do.  Default 1. */
int kh_bsgs_set_bloom_multiplier(kh_ctx *ctx, uint32_t mult);
int kh_bsgs_setup(kh_ctx *ctx, uint64_t n, uint64_t k, kh_bsgs_info *info);
/* after kh_bsgs_setup: the device bytes this context holds once its tables are built and it scans
 * (the three layers, the bP rows, the inversion pad of the giant walk, lane state, candidate buffers
 * at their current size, a kh_bsgs_scan_list of up to 2^16 bases), and how many of them it holds
 * already.  A lower bound: longer lists (32 B per base) and candidate buffers grown on overflow come
 * on top.  The pad counted is the 2^18-lane one (8 GB); a call of >= 2^21 walk groups widens it to
 * 2^21 lanes (64 GB; 2^20: 32 GB) only while 32 GB of the device stay free after it */
int kh_bsgs_memory(kh_ctx *ctx, uint64_t *needed_bytes, uint64_t *held_bytes);
int kh_bsgs_build(kh_ctx *ctx);                  /* baby-step blooms + sorted bP table on the GPU */
/* -S table files in the reference's formats (keyhunt.cpp:2504-2652 write, 1983-2230 read), in dir
 * (NULL -> "."): keyhunt_bsgs_4_<M>.blm, keyhunt_bsgs_6_<M2>.blm, keyhunt_bsgs_7_<M3>.blm (256 x
 * {struct bloom, bits, sha256 x2}) and keyhunt_bsgs_2_<M3>.tbl (sorted 16-byte rows + sha256).
 * Files are byte-identical to the reference's except the heap pointer it stores in each struct
 * bloom.  kh_bsgs_save needs kh_bsgs_build (or _load) first; with the blocked layer 1 it builds the
 * reference-layout layer 1 for the file.  kh_bsgs_load replaces kh_bsgs_build after kh_bsgs_setup;
 * with the blocked layout it checks the layer-1 file and rebuilds the blocked layer on the GPU. */
#define KH_LOAD_SKIP_CHECKSUM 1   /* the reference's -6 */
int kh_bsgs_save(kh_ctx *ctx, const char *dir);
int kh_bsgs_load(kh_ctx *ctx, const char *dir, uint32_t flags);

/* -S for -m address|rmd160|xpoint (and -c eth): the target file cache data_<hex>.dat, named by the
 * CLI from the first 4 bytes of the target file's sha256 (keyhunt.cpp:7043-7049).  Layout:
 * sha256(bloom bits) | struct bloom (112 B) | bloom bits | sha256(rows) | u64 row bytes | sorted
 * 20-byte rows.  kh_targets_save writes the context's targets (after kh_set_targets), replacing
 * writeFileIfNeeded (keyhunt.cpp:7756-7855); kh_targets_load stands in for kh_set_targets and takes
 * the bloom geometry and bits from the file, as readFileAddress does (keyhunt.cpp:7033-7210), so a
 * file the reference wrote probes identically.  flags: KH_LOAD_SKIP_CHECKSUM. */
int kh_targets_save(kh_ctx *ctx, const char *path);
int kh_targets_load(kh_ctx *ctx, const char *path, uint32_t flags);
/* targets: n x {x[32], y[32]} affine points (big-endian) */
int kh_bsgs_set_targets(kh_ctx *ctx, const uint8_t *xy, uint32_t n);
/* Walk n_bases bases start, start + 2N, ... for every target not yet found.  Keys already found
 * are skipped (like bsgs_found[]).  found: keys found by THIS call.  With one target, a call that
 * starts at the base after the previous call's last one (same n_bases) continues its lanes. */
int kh_bsgs_scan(kh_ctx *ctx, const uint8_t start[32], uint64_t n_bases, kh_bsgs_found *found, uint32_t cap,
                 uint32_t *n_found);
/* Same for an arbitrary list of bases (n_bases x 32-byte big-endian keys), e.g. the -B backward /
 * both / random / dance schedules (keyhunt.cpp:5953, 6211, 4893, 5674): each base walks its own
 * 2N keys exactly as in kh_bsgs_scan. */
int kh_bsgs_scan_list(kh_ctx *ctx, const uint8_t *bases, uint64_t n_bases, kh_bsgs_found *found, uint32_t cap,
                      uint32_t *n_found);
int kh_bsgs_reset_found(kh_ctx *ctx);
/* first-level bloom candidates seen so far (for stats / parity tests) */
int kh_bsgs_candidates(kh_ctx *ctx, uint64_t *count);
/* first-level candidates and layer-2 hits of their second checks (bsgs_secondcheck's bloom_check
 * positives, keyhunt.cpp:5177-5180) since kh_bsgs_setup.  The second check runs on the GPU
 * (k_refine) unless the environment sets KH_REFINE=host at kh_open; both give the same counts. */
int kh_bsgs_refine_stats(kh_ctx *ctx, uint64_t *first_level, uint64_t *second_level);

/* ---- measurement -------------------------------------------------------------------------- */
/* Accumulated device time of walk launches of one kind since the last reset, measured with
 * HIP events on the context's stream.  kind: 0 address/rmd160, 1 xpoint, 2 bsgs giant,
 * 3 bsgs build, 4 lane setup (scalar mult). */
int kh_kernel_time(kh_ctx *ctx, uint32_t kind, uint64_t *launches, double *ms, uint64_t *points);
int kh_kernel_time_reset(kh_ctx *ctx);

/* ---- parity hooks (used by tests/) -------------------------------------------------------- */
/* k*G for n scalars (big-endian 32 B each) -> n x {x,y} (big-endian), through the lane-setup kernel */
int kh_pubkeys(kh_ctx *ctx, const uint8_t *scalars, uint32_t n, uint8_t *xy);
/* X (and Y if out_y) of points start + i*stride, i < n_points (multiple of 1024), via the walk */
int kh_walk_points(kh_ctx *ctx, const uint8_t start[32], const uint8_t stride[32], uint64_t n_points,
                   uint8_t *out_x, uint8_t *out_y);
/* per input point: hash160(02||X), hash160(03||X), hash160(04||X||Y) -> 60 bytes */
int kh_hash160(kh_ctx *ctx, const uint8_t *xy, uint32_t n, uint8_t *out60);
/* field ops on the device: per pair (a,b) -> mul, sqr(a), inv(a), add, sub (5 x 32 B) */
int kh_field_ops(kh_ctx *ctx, const uint8_t *a, const uint8_t *b, uint32_t n, uint8_t *out160);
/* bloom_check of n items (len 20 or 32) against the target bloom (layer 0) or BSGS layer 1..3 */
int kh_bloom_check(kh_ctx *ctx, uint32_t layer, const uint8_t *items, uint32_t n, uint32_t len, uint8_t *out);
/* copy a bloom back: layer 0 = target bloom, 1..3 = BSGS layers (256 shards concatenated, unpadded) */
int kh_get_bloom(kh_ctx *ctx, uint32_t layer, uint8_t *buf, uint64_t cap, uint64_t *bytes);
/* The context's own sorted bP rows (16 B each, the reference's bsgs_xvalue layout), valid until the
 * next kh_bsgs_build / _load / _set_table / kh_close: --ptable writes them to its file without a copy. */
int kh_bsgs_table_rows(kh_ctx *ctx, const uint8_t **rows, uint64_t *n_rows);

/* Memory-mapped bloom files (--mapped, keyhunt.cpp:724-806, 7630-7706; bloom/bloom.cpp:491-747): the
 * file is the raw bit array of a filter whose geometry the reference derives from the entry count or,
 * when it reloads an existing file, from the file size (bits = bytes * 8).
 * kh_bloom_add: bloom_add of n items of len bytes (20, a shorter hash160 prefix, or 32) into the flat
 * bit array bf of that geometry (host only, no GPU).
 * kh_bsgs_layer_bits: after kh_bsgs_build / _load, OR the baby-step X's of layer 1, 2 or 3 (the first
 * M, M2 or M3 babies) into 256 contiguous shards of bytes each, with the given bits and hashes. */
int kh_bloom_add(uint8_t *bf, uint64_t bits, uint32_t hashes, const uint8_t *items, uint64_t n, uint32_t len);
int kh_bsgs_layer_bits(kh_ctx *ctx, uint32_t layer, uint64_t bits, uint32_t hashes, uint64_t bytes, uint8_t *shards);

/* bsgsd semantics (bsgsd.cpp:2544-2561): the daemon's worker also tests every base point against the
 * target, so a key that is exactly a base (offset 0, which the giant/baby steps reach only through the
 * point at infinity) is found there; keyhunt's own worker (keyhunt.cpp:4625-4640) has no such test and
 * misses it.  Off by default (the CLI's behaviour); bsgsd-amd turns it on. */
int kh_bsgs_set_base_check(kh_ctx *ctx, int enable);

/* Parity hook: with logging enabled (cleared on every call), kh_bsgs_scan / _list record every
 * first-level candidate -- layer-1 bloom positive, keyhunt.cpp:4819-4823 -- as (base ordinal within
 * its call, giant index a = 1024 j + i within the base, layer-2 mask of its second check), in
 * giant-step order per round.  kh_bsgs_get_candidates copies up to cap of them. */
int kh_bsgs_log_candidates(kh_ctx *ctx, int enable);
int kh_bsgs_get_candidates(kh_ctx *ctx, uint64_t *base_index, uint32_t *a, uint32_t *mask, uint64_t cap,
                           uint64_t *n);
/* bsgs_secondcheck's layer-2 hit mask for n base keys (32-byte big-endian each) against target
 * `target`, from the GPU kernel (k_refine) and from the host code: bit i set when the point
 * Q - base_key*G + AMP2[i] passes bloom_bPx2nd (keyhunt.cpp:5151-5184) */
int kh_bsgs_second_masks(kh_ctx *ctx, uint32_t target, const uint8_t *base_keys, uint32_t n, uint32_t *gpu_mask,
                         uint32_t *host_mask);
/* sorted bP table as the reference's 16-byte bsgs_xvalue rows {value[6], pad[2], index u64 LE} */
int kh_get_bsgs_table(kh_ctx *ctx, uint8_t *buf, uint64_t cap_rows, uint64_t *rows);
/* --ptable FILE --load-ptable (keyhunt.cpp:1847-1956): after kh_bsgs_build (or _load), replace the
 * sorted bP table with n_rows = M3 rows of the same 16-byte layout taken from the reference's raw
 * table file.  The rows are used as given, as the reference's read-only mapping is. */
int kh_bsgs_set_table(kh_ctx *ctx, const uint8_t *rows, uint64_t n_rows);

#ifdef __cplusplus
}
#endif
#endif /* KH_GPU_H */
