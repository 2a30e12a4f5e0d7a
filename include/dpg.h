/*
 * dpg.h -- C ABI of the MI355X-native DPEngine.aggregate hot path
 *          (libdpg.so, built from the HIP sources in pipelinedp_amd/csrc for gfx950).
 *
 * Plain pointers and sizes only; no torch or HIP types in the signatures
 * (streams travel as void*).  Every entry point returns an int status
 * (DPG_OK = 0) and never throws across the ABI; dpg_last_error() returns
 * the message of the last failure on a context.  One context per
 * (host thread, device); calls on one context are not re-entrant.
 *
 * Reference interfaces each entry point replaces (paths relative to the
 * PipelineDP reference tree):
 *   dpg_bound_aggregate  <- DPEngine._aggregate up to the partition merge:
 *        pipeline_dp/dp_engine.py:113-151 (extract, drop public, bound,
 *        drop pid, add empty public, combine_accumulators_per_key), i.e.
 *        contribution_bounders.py:66-195 + combiners.py:691-706 +
 *        pipeline_backend.py:531-565 (LocalBackend sample/group/reduce).
 *   dpg_select_and_noise <- DPEngine._select_private_partitions_internal
 *        (dp_engine.py:305-361, PyDP create_partition_strategy().should_keep)
 *        fused with CompoundCombiner.compute_metrics (combiners.py:708-730,
 *        dp_computations.py:120-184, 307-366, 541-576; PyDP add_noise).
 *   dpg_compact_kept     <- the LocalBackend `filter` materialisation
 *        (pipeline_backend.py:514-515) of the selected partitions.
 *   dpg_preaggregate     <- utility analysis' per-(privacy id, partition)
 *        pre-aggregation: analysis/contribution_bounders.py:37-77
 *        (AnalysisContributionBounder) and analysis/pre_aggregation.py:19-61.
 *   dpg_utility_analysis <- the per-partition utility combiners of every
 *        configuration of a sweep: analysis/per_partition_combiners.py:195-356
 *        (PartitionSelection / Sum / Count / PrivacyIdCount / RawStatistics)
 *        with analysis/poisson_binomial.py:39-83, driven by
 *        analysis/utility_analysis_engine.py:98-143.
 *   dpg_dataset_histograms <- pipeline_dp/dataset_histograms/
 *        computing_histograms.py:420-474 (compute_dataset_histograms, over
 *        the dpg_preaggregate pairs) and :642-684
 *        (compute_dataset_histograms_on_preaggregated_data), which feed
 *        DPEngine.calculate_private_contribution_bounds (dp_engine.py:432-484)
 *        and analysis/parameter_tuning.py:278-348 (tune).
 */
#ifndef DPG_H_
#define DPG_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ---- */
#define DPG_OK 0
#define DPG_ERR_INVALID_ARG 1
#define DPG_ERR_KEY_RANGE 2   /* pid outside its declared range or pk outside [0, P) */
#define DPG_ERR_HIP 3
#define DPG_ERR_OOM 4
#define DPG_ERR_UNSUPPORTED 5

/* ---- Philox key tags: domain separation of the keyed random streams ---- */
#define DPG_TAG_PAIR 0x50414952u   /* pair priority      (pid, pk)              */
#define DPG_TAG_REC 0x52454344u    /* record priority    (pid, pk, record id)   */
#define DPG_TAG_SELECT 0x53454C45u /* partition selection (pk)                  */
#define DPG_TAG_NOISE 0x4E4F4953u  /* metric noise        (pk, slot)            */

/* ---- contribution-bounding modes (dp_engine.py:370-382) ---- */
#define DPG_MODE_CROSS_AND_PER_PARTITION 0 /* SamplingCrossAndPerPartition   */
#define DPG_MODE_PER_PRIVACY_ID 1          /* SamplingPerPrivacyId (L1)      */
#define DPG_MODE_CROSS_PARTITION 2         /* SamplingCrossPartition         */

/* ---- how SUM is bounded (combiners.py:348-353) ---- */
#define DPG_SUM_NONE 0
#define DPG_SUM_CLIP_VALUE 1     /* clip every value to [min_value, max_value] */
#define DPG_SUM_CLIP_PARTITION 2 /* clip the per-(pid,pk) sum                   */

/* ---- accumulator mask ---- */
#define DPG_M_COUNT 1u
#define DPG_M_SUM 2u
#define DPG_M_PRIVACY_ID_COUNT 4u
#define DPG_M_MEAN 8u
#define DPG_M_VARIANCE 16u

/* ---- partition selection (partition_selection.py:19-44) ---- */
#define DPG_SELECT_NONE 0 /* public partitions: keep iff in public_mask */
#define DPG_SELECT_TRUNCATED_GEOMETRIC 1
#define DPG_SELECT_LAPLACE_THRESHOLD 2
#define DPG_SELECT_GAUSSIAN_THRESHOLD 3

/* ---- noise ---- */
#define DPG_NOISE_NONE 0
#define DPG_NOISE_LAPLACE 1
#define DPG_NOISE_GAUSSIAN 2

#define DPG_FAMILY_SCALAR 0   /* Count / Sum / PrivacyIdCount combiners    */
#define DPG_FAMILY_MEAN 1     /* MeanCombiner (+ PrivacyIdCount)           */
#define DPG_FAMILY_VARIANCE 2 /* VarianceCombiner (+ PrivacyIdCount)       */

/* noise slots (each gets its own Philox counter) */
#define DPG_SLOT_COUNT 0
#define DPG_SLOT_SUM 1 /* SUM, or the normalised sum of MEAN/VARIANCE */
#define DPG_SLOT_NSQ 2 /* normalised sum of squares (VARIANCE)        */
#define DPG_SLOT_PID 3 /* PRIVACY_ID_COUNT                             */

/* value-vector entries an output column can be mapped from */
#define DPG_V_COUNT 0
#define DPG_V_SUM 1
#define DPG_V_MEAN 2
#define DPG_V_VARIANCE 3
#define DPG_V_PRIVACY_ID_COUNT 4

typedef struct dpg_bound_params {
    int32_t mode;        /* DPG_MODE_*                               */
    int32_t sum_mode;    /* DPG_SUM_*                                */
    uint32_t metric_mask;/* DPG_M_* accumulators to produce          */
    int32_t reserved0;
    int64_t max_partitions_contributed;      /* mpc (l0)            */
    int64_t max_contributions_per_partition; /* mcpp (linf)         */
    int64_t max_contributions;               /* L1 (PER_PRIVACY_ID) */
    double min_value, max_value;
    double min_sum_per_partition, max_sum_per_partition;
    int64_t n_partitions;        /* P: pk ids are dense in [0, P)   */
    const uint8_t *public_mask;  /* bitmap of P bits (device memory for
                                    libdpg, host memory for the oracle);
                                    NULL = private partition selection */
    int64_t pid_min;             /* privacy ids lie in [pid_min,        */
    int64_t pid_count;           /*   pid_min + pid_count); pid_count <= 2^32.
                                    0 = unknown: libdpg reduces min/max on
                                    the device first                     */
    int64_t rec_id_offset;       /* global id of input record 0: the
                                    record sampler is keyed by
                                    (pid, pk, rec_id_offset + i), so shards
                                    of one dataset sample as the whole   */
    uint64_t nonce;              /* per-release nonce: every keyed stream of
                                    the call uses dpg_stream_seed(ctx seed,
                                    nonce).  Callers pass a FRESH random
                                    nonce per release (the reference draws
                                    fresh randomness per call,
                                    dp_computations.py:131-133, 151-152,
                                    pipeline_backend.py:540-544) and the
                                    same nonce on every rank of one release */
} dpg_bound_params;

/* Dense per-partition partial accumulators (structure of arrays).
 * rows  = number of kept (privacy id, partition) pairs = privacy id count
 * count = number of kept records; sum = bounded sum;
 * nsum  = sum(clip(v) - mid), nsq = sum((clip(v) - mid)^2)
 * Unused float arrays may be NULL. */
typedef struct dpg_partials {
    int64_t n_partitions;
    int64_t *rows;
    int64_t *count;
    double *sum;
    double *nsum;
    double *nsq;
} dpg_partials;

typedef struct dpg_select_params {
    int32_t strategy;            /* DPG_SELECT_*                          */
    int32_t table_len;           /* truncated geometric: len(keep_table)  */
    const double *keep_table;    /* host pointer; pi(n) for n < table_len,
                                    1.0 beyond                              */
    double threshold;            /* Laplace/Gaussian thresholding          */
    double noise_scale;          /* b (Laplace) or sigma (Gaussian)        */
    int64_t pre_threshold;       /* 0 = none                               */
    int64_t max_rows_per_privacy_id; /* dp_engine.py:156-164 (normally 1)  */
    int64_t pk_offset;           /* global pk id of partials index 0       */
    const uint8_t *public_mask;  /* DPG_SELECT_NONE: keep iff bit set
                                    (indexed by local partition id)        */
    uint64_t nonce;              /* per-release nonce of the selection and
                                    noise draws (see dpg_bound_params)      */
    int64_t pk_stride;           /* global pk of partials index i is
                                    pk_offset + i * pk_stride (multi-GPU
                                    slices are interleaved: rank r owns
                                    r, r + R, ...); <= 0 means 1            */
} dpg_select_params;

typedef struct dpg_noise_params {
    int32_t noise_kind;  /* DPG_NOISE_*                                  */
    int32_t family;      /* DPG_FAMILY_*                                 */
    uint32_t slot_mask;  /* bit s: slot s exists (SCALAR / pid slot)     */
    int32_t n_outputs;   /* output columns per partition                 */
    int32_t out_src[8];  /* column j <- value vector entry DPG_V_*       */
    double scale[4];     /* per-slot noise scale: b or sigma             */
    double mid;          /* MEAN/VARIANCE range middle                   */
    int32_t mean_const;  /* VARIANCE: min_value == max_value             */
    int32_t msq_const;   /* VARIANCE: squares interval degenerate        */
    double mean_const_value;
    double msq_const_value;
} dpg_noise_params;

/* One (privacy id, partition) pair of the utility-analysis pre-aggregate
 * (24 bytes): the pair's record count and value sum, the number of
 * partitions its privacy id contributes to and the privacy id's records.
 * Bit 31 of contributions_leader is the leader flag (dpg_preaggregate sets
 * it on one pair per privacy id); bits 0-30 are n_contributions. */
typedef struct dpg_pair_entry {
    uint32_t pk;
    uint32_t count;
    double sum;
    uint32_t n_partitions;
    uint32_t contributions_leader;  /* n_contributions | leader << 31 */
} dpg_pair_entry;

/* One row of a MultiParameterConfiguration (analysis/data_structures.py
 * :24-103) with the budget of its mechanisms resolved. */
typedef struct dpg_ua_config {
    int64_t max_partitions_contributed;      /* l0                          */
    int64_t max_contributions_per_partition; /* linf of COUNT               */
    double min_sum_per_partition;            /* SUM clipping                */
    double max_sum_per_partition;
    int32_t selection_strategy;  /* DPG_SELECT_* (private partitions)      */
    int32_t reserved;
    int64_t pre_threshold;       /* 0 = none                               */
    const double *keep_table;    /* host: truncated geometric pi(n)        */
    int64_t table_len;
    double threshold;            /* Laplace / Gaussian thresholding        */
    double noise_scale;
    double noise_std[3];         /* report: noise std of SUM, COUNT and
                                    PRIVACY_ID_COUNT (compute_dp_count_noise_std,
                                    dp_computations.py:369-395)             */
} dpg_ua_config;

typedef struct dpg_ua_params {
    int32_t n_configs;           /* 1..64                                   */
    uint32_t metric_mask;        /* DPG_M_SUM | DPG_M_COUNT | DPG_M_PRIVACY_ID_COUNT */
    int32_t public_partitions;   /* 1: public partitions (no selection)    */
    int32_t reserved;
    const dpg_ua_config *configs;/* host [n_configs]                       */
    const uint8_t *sample_mask;  /* device bitmap of the partitions kept by
                                    partitions_sampling_prob, or NULL       */
    const uint8_t *public_mask;  /* device bitmap of public partitions     */
} dpg_ua_params;

/* Dataset histograms (pipeline_dp/dataset_histograms/histograms.py:60-75).
 * Integer histograms (L0, L1, LINF, COUNT_PER_PARTITION,
 * PRIVACY_ID_PER_PARTITION, in this order) have DPG_HIST_INT_BINS bins of 3
 * significant digits: bin v for v < 1000 ([v, v+1)), else
 * 1000 + 900 e + (m - 100) for [m 10^(e+1), (m+1) 10^(e+1)), m in [100, 999].
 * LINF_SUM has DPG_HIST_SUM_BINS equal bins between the smallest and the
 * largest pair sum; lowers[i] = np.linspace(min, max, bins + 1)[i]. */
#define DPG_HIST_INT_BINS 16300
#define DPG_HIST_SUM_BINS 10000
#define DPG_HIST_L0 0
#define DPG_HIST_L1 1
#define DPG_HIST_LINF 2
#define DPG_HIST_COUNT_PER_PARTITION 3
#define DPG_HIST_PRIVACY_ID_PER_PARTITION 4

typedef struct dpg_hist_out {
    uint64_t *int_bins;  /* device [5][DPG_HIST_INT_BINS][3]: count, sum, max;
                            a bin exists iff count > 0 or max > 0            */
    uint64_t *sum_count; /* device [DPG_HIST_SUM_BINS] LINF_SUM counts       */
    double *sum_sum;     /* device [DPG_HIST_SUM_BINS] LINF_SUM sums         */
    double *sum_max;     /* device [DPG_HIST_SUM_BINS] LINF_SUM maxima       */
    double *lowers;      /* device [DPG_HIST_SUM_BINS + 1] LINF_SUM lowers   */
} dpg_hist_out;

typedef struct dpg_ctx dpg_ctx;

/* Context: device ordinal and the 64-bit seed of every keyed random stream.
 * Returns NULL on failure. */
dpg_ctx *dpg_ctx_create(int device, uint64_t seed);
void dpg_ctx_destroy(dpg_ctx *ctx);
int dpg_last_error(dpg_ctx *ctx, char *buf, size_t len);
int dpg_set_seed(dpg_ctx *ctx, uint64_t seed);

/* The 64-bit key of every keyed random stream of one release:
 * mix64(seed ^ mix64(nonce + 0x9E3779B97F4A7C15)) with mix64 the SplitMix64
 * finaliser.  Two releases with different nonces draw independent sampling,
 * selection and noise; the same (seed, nonce) reproduces a release exactly
 * (tests, and every rank of one multi-GPU release). */
uint64_t dpg_stream_seed(uint64_t seed, uint64_t nonce);

/* Tuning / testing hook: average records per fine privacy-id bucket the
 * partition levels aim for (default 256; smaller values force more levels on
 * small inputs) and the chunk capacity, i.e. the most records bounded
 * together in LDS (default and maximum 1024; chunks of <= min(cap, 512)
 * records run one wave each, larger ones one 256-thread workgroup).  Buckets
 * over the capacity are split by further privacy-id hash bits; a bucket
 * still over it takes the global-memory path.  <= 0 keeps the current
 * value. */
int dpg_set_tuning(dpg_ctx *ctx, int32_t bucket_target, int32_t bucket_cap);

/* Contribution bounding + per-(pid,pk) accumulators + merge per partition.
 * pid, pk: device int64[n]; value: device double[n] or NULL (COUNT / PID
 * only).  out->* device arrays of out->n_partitions entries; they are
 * zero-filled by the call.  stream: hipStream_t or NULL. */
int dpg_bound_aggregate(dpg_ctx *ctx, const int64_t *pid, const int64_t *pk,
                        const double *value, int64_t n,
                        const dpg_bound_params *params, dpg_partials *out,
                        void *stream);

/* Partition selection + noise over dense partials (device arrays).
 * keep: device uint8[P]; out: device double[P * noise->n_outputs]. */
int dpg_select_and_noise(dpg_ctx *ctx, const dpg_partials *partials,
                         const dpg_select_params *select,
                         const dpg_noise_params *noise, uint8_t *keep,
                         double *out, void *stream);

/* Stream compaction of the kept partitions: writes the kept local ids to
 * kept_ids (device int64[P]) and their output rows to kept_out (device
 * double[P * n_outputs]); *n_kept (host) receives the count (synchronises
 * the stream). */
int dpg_compact_kept(dpg_ctx *ctx, const uint8_t *keep, const double *out,
                     int64_t n_partitions, int32_t n_outputs,
                     int64_t *kept_ids, double *kept_out, int64_t *n_kept,
                     void *stream);

/* The same without the host synchronisation: info (device int64[2])
 * receives the kept count (info[0]) and the bounding's error bits (info[1];
 * bit 1: the internal hash-table error dpg_compact_kept reports), in stream
 * order, so that a caller can enqueue the next release before reading them. */
int dpg_compact_kept_async(dpg_ctx *ctx, const uint8_t *keep, const double *out,
                           int64_t n_partitions, int32_t n_outputs,
                           int64_t *kept_ids, double *kept_out, int64_t *info,
                           void *stream);

/* Utility-analysis pre-aggregate: no contribution bounding; one entry per
 * distinct (privacy id, partition) pair, sorted by partition key, into
 * pairs[0, *n_pairs) (device, `capacity` entries; n always suffices), and
 * partition_start (device int64[P + 1]): the pairs of partition k are
 * [partition_start[k], partition_start[k + 1]).  Of *p only n_partitions,
 * public_mask (pairs of other partitions are dropped first), pid_min,
 * pid_count and rec_id_offset are used.  value may be NULL (sums 0).
 * n < 2^31 (else DPG_ERR_UNSUPPORTED).  *n_pairs (host) receives the pair count (synchronises the stream); if it
 * exceeds capacity the call fails with DPG_ERR_INVALID_ARG. */
int dpg_preaggregate(dpg_ctx *ctx, const int64_t *pid, const int64_t *pk, const double *value,
                     int64_t n, const dpg_bound_params *p, dpg_pair_entry *pairs,
                     int64_t capacity, int64_t *partition_start, int64_t *n_pairs,
                     void *stream);

/* Per-partition utility analysis of up to 64 configurations in one pass
 * over the sorted pre-aggregate.  Device outputs:
 *   raw    double[P][2]: privacy id count, count (RawStatistics)
 *   errors double[P][M][5][C], M = metrics present in the order SUM, COUNT,
 *          PRIVACY_ID_COUNT; the 5 fields are sum, clipping_to_min_error,
 *          clipping_to_max_error, expected_l0_bounding_error and the l0
 *          bounding variance (SumMetrics before the noise std is attached)
 *   keep   double[P][C]: partition_selection_probability_to_keep (NULL for
 *          public partitions)
 *   report double[29][F][C] or NULL: the cross-partition combine
 *          (analysis/cross_partition_combiners.py:264-343) summed per
 *          partition-size bucket (utility_analysis.py:29-39, 182-251), F =
 *          4 + 24 M fields: partitions, weight, 2 partition-info terms, then
 *          per metric its sum, 3 data-drop terms and 10 absolute + 10
 *          relative error terms, weighted by the keep probability; dividing
 *          by the weight / metric sums gives the UtilityReport
 *   *n_out (host, optional) receives the number of output partitions.
 * Partitions outside sample_mask or without pairs (and not public) stay 0
 * and are not in the output. */
int dpg_utility_analysis(dpg_ctx *ctx, const dpg_pair_entry *pairs,
                         const int64_t *partition_start, int64_t n_partitions,
                         const dpg_ua_params *params, double *raw, double *errors, double *keep,
                         double *report, int64_t *n_out, void *stream);

/* Dataset histograms over a pre-aggregate sorted by partition key (pairs,
 * partition_start as dpg_preaggregate writes them).  pre_aggregated = 0:
 * the pairs come from dpg_preaggregate, whose leader bit marks one pair per
 * privacy id (the per-privacy-id histograms count those); 1: user-supplied
 * (count, sum, n_partitions, n_contributions) rows, L0 / L1 weighted by
 * 1 / n_partitions per exact value and rounded half to even
 * (computing_histograms.py:81-102, 482-529).  All outputs are device
 * arrays, zero-filled by the call. */
int dpg_dataset_histograms(dpg_ctx *ctx, const dpg_pair_entry *pairs, int64_t n_pairs,
                           const int64_t *partition_start, int64_t n_partitions,
                           int32_t pre_aggregated, const dpg_hist_out *out, void *stream);

/* ---- multi-GPU: an RCCL communicator for the partial merge ----
 * One process per GPU, records sharded by privacy id (bounding is then
 * shard-local).  Rank 0 calls dpg_comm_unique_id; the
 * DPG_COMM_ID_BYTES bytes reach every rank by the host's own means (MPI,
 * TCP, a shared file); each rank then attaches a communicator to its
 * context.  RCCL is loaded on first use (dlopen of librccl), so libdpg.so
 * has no link-time dependency on it and shares the copy a host such as
 * PyTorch has already loaded.  Replaces the reference's shuffle of
 * (partition key, accumulator) pairs between workers
 * (pipeline_backend.py:712-823, combine_accumulators_per_key on Beam/Spark). */
#define DPG_COMM_ID_BYTES 128
int dpg_comm_unique_id(uint8_t *id);
int dpg_ctx_create_comm(dpg_ctx *ctx, const uint8_t *id, int rank, int nranks);
/* Partition ownership is interleaved: rank r owns the partitions
 * r, r + R, r + 2R, ... (R = nranks), so hot low partition ids spread over
 * every rank; slice element i is partition lo + i * R with lo = r.
 * The merge also carries each rank's internal-error flag (a bounding whose
 * hash table overflowed, dpg_compact_kept's error): every rank receives the
 * sum of all flags and latches it, so a failure on any rank fails the
 * dpg_compact_kept of every rank instead of releasing partials of a
 * mis-bounded shard.
 *
 * dpg_reduce_scatter_partials sums the dense partials of every rank (ONE
 * ncclReduceScatter of all non-null arrays packed as float64 -- exact below
 * 2^53) and writes this rank's slice (n = number of partitions = r mod R
 * in [0, P)) into `slice` (its arrays hold >= S = ceil(P / R) entries; the
 * same arrays non-null as in `full`; slice->n_partitions is set to n).
 * Stream-ordered on `stream`. */
int dpg_reduce_scatter_partials(dpg_ctx *ctx, const dpg_partials *full, dpg_partials *slice,
                                int64_t *lo, int64_t *n, void *stream);
/* The same merge with the host's own collective (MPI, gloo, a TCP ring):
 * dpg_pack_partials writes the non-null arrays of `full` as float64 in the
 * reduce-scatter layout pack[rank][B], B = arrays * S + 1: [array][S] with
 * element i = partition i * R + rank (zero past P; array order rows, count,
 * sum, nsum, nsq), then this rank's error flag (pack holds nranks * B
 * doubles); after the host's element-wise sum over ranks delivers this
 * rank's block part[B], dpg_unpack_partials writes it into `slice` (its
 * non-null arrays name the packed ones), latches a nonzero error sum and
 * returns lo = rank and n.  Stream-ordered on `stream`. */
int dpg_pack_partials(dpg_ctx *ctx, const dpg_partials *full, int nranks, double *pack,
                      void *stream);
int dpg_unpack_partials(dpg_ctx *ctx, const double *part, int64_t n_partitions, int nranks,
                        int rank, dpg_partials *slice, int64_t *lo, int64_t *n, void *stream);
/* The error flag alone, for a merge the host routes itself (e.g. a sparse
 * all-to-all of the occupied partitions): dpg_export_error writes 1.0 to
 * device *dst if the context's last bounding latched an internal error, else
 * 0.0; dpg_import_error latches the error if any of the n device doubles at
 * src is nonzero.  Both stream-ordered, no host synchronisation. */
int dpg_export_error(dpg_ctx *ctx, double *dst, void *stream);
int dpg_import_error(dpg_ctx *ctx, const double *src, int64_t n, void *stream);

/* Timing/profiling aid: per-stage device time (ms) of the last
 * dpg_bound_aggregate / dpg_preaggregate / dpg_dataset_histograms call,
 * measured with HIP events on its stream (waits for the last event).
 * names (comma separated, <= names_len bytes): e.g. "begin",
 * "partition1:hist", "partition1:scatter", "partition2:hist",
 * "partition2:scatter", "chunks", "bound.kernel=sort" (zero-length marker
 * of the small-chunk kernel that ran), "bound", "bound.wide" (sort kernel:
 * chunks of more than 256 candidates), "bound.medium", "bound.tail",
 * "items:hist", "items:scatter", "reduce". */
int dpg_last_stage_times(dpg_ctx *ctx, char *names, size_t names_len,
                         double *ms, int32_t max_stages, int32_t *n_stages);

#ifdef __cplusplus
}
#endif
#endif /* DPG_H_ */
