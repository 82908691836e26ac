/*
 * sift_hip.h — C-ABI boundary of the MI355X-native SIFT extractor.
 *
 * This is the thin shim that sits directly under the reference's public
 * entry point
 *     std::vector<Keypoint> detect_keypoints_and_descriptors(const Image&, ...)
 * (reference src/sift.hh:65-71, implemented at src/sift.cpp:712-776).
 * The C++ drop-in (sift.hh / libsift_amd.so) wraps these calls and rethrows
 * failures as std::runtime_error, the reference's error convention
 * (src/image.cpp:43,159,222, src/image_io.cpp:24,149).
 *
 * Plain pointers and sizes only: no torch, no C++ types, no HIP types in the
 * signatures (streams are passed as opaque void*).
 *
 * All status codes: 0 = success, negative = error (see sift_hip_strerror).
 */
#ifndef SIFT_HIP_H
#define SIFT_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SIFT_HIP_ABI_VERSION 3

/* ---- status codes ------------------------------------------------------ */
#define SIFT_OK 0
#define SIFT_ERR_ARG -1          /* bad argument (null pointer, bad size)     */
#define SIFT_ERR_CHANNELS -2     /* channels not in {1,3}: reference reads
                                    past the pixel for c=2 (image.cpp:16-18)  */
#define SIFT_ERR_TOO_SMALL -3    /* min(W0,H0)/3 == 0: the reference takes
                                    log2(0) (sift.cpp:134), undefined         */
#define SIFT_ERR_HIP -4          /* a HIP runtime call failed                  */
#define SIFT_ERR_NOMEM -5        /* device or host allocation failed           */
#define SIFT_ERR_NO_DEVICE -6    /* no HIP device / bad device index           */
#define SIFT_ERR_PARAM -7        /* parameter outside the supported range      */
#define SIFT_ERR_STATE -8        /* call order violated (e.g. no prior detect) */
#define SIFT_ERR_NO_COMM -9      /* RCCL missing or a collective failed        */
#define SIFT_ERR_PEER -10        /* another rank of a collective failed; this
                                    rank joined every collective and returns */

/*
 * Parameters of detect_keypoints_and_descriptors (reference sift.hh:65-71),
 * same names, same defaults (see sift_params_default), plus two extensions:
 *   max_octaves        0 = the reference formula floor(log2(min(W0,H0)/3))
 *                      (sift.cpp:132-137); >0 caps the octave count
 *                      (needed for BASELINE config 3, "5 octaves").
 *   write_keypoints_png reserved for the reference's keypoints.png side effect
 *                      (sift.cpp:765-768); the C-ABI never writes files, the
 *                      C++ drop-in honours it.
 * num_bins is a double in the reference API and is narrowed to int by
 * compute_orientations (sift.cpp:450); it is narrowed the same way here.
 */
typedef struct sift_params {
    int double_image_size;      /* true  */
    int intervals;              /* 3     */
    int window_size;            /* 3     */
    int max_octaves;            /* 0 (extension) */
    double init_sigma;          /* 1.6   */
    double contrast_threshold;  /* 0.04  */
    double eigen_ratio;         /* 10.0  */
    double num_bins;            /* 36    */
    double peak_ratio;          /* 0.8   */
    double ori_sigma_factor;    /* 1.5   */
    double desc_scale_factor;   /* 3.0   */
    int write_keypoints_png;    /* 0 in the C-ABI (extension) */
    int reserved;
} sift_params;

/*
 * One keypoint record. Layout-identical to the reference struct Keypoint
 * (sift.hh:15-23): x@0 y@8 octave@16 layer@20 size@24 pori@32 desc@40,
 * sizeof == 168, so a sift_kp array can be memcpy'd into
 * std::vector<Keypoint> storage.
 */
typedef struct sift_kp {
    double x;
    double y;
    int octave;
    int layer;
    double size;
    double pori;
    uint8_t desc[128];
} sift_kp;

/* Candidate extremum (x, y, DoG layer z, octave) — reference tuple
 * Extrema (sift.cpp:14), with x,y stored as ints (they are integral). */
typedef struct sift_extremum {
    int x;
    int y;
    int z;
    int octave;
} sift_extremum;

typedef struct sift_ctx sift_ctx;

/* Fill *p with the reference defaults (sift.hh:65-71). */
void sift_params_default(sift_params* p);

/* Create a context bound to HIP device `device`: owns four HIP streams and
 * SIFT_MAX_INFLIGHT job slots, each with a device arena that grows to the
 * largest job seen. */
int sift_hip_create(int device, sift_ctx** out);
int sift_hip_destroy(sift_ctx* ctx);

/*
 * Full pipeline on one image (reference sift.cpp:712-776 minus the PNG side
 * effect). `hwc` is the reference Image buffer: interleaved HWC doubles,
 * data[(y*w+x)*c+ch] (image_io.cpp:81-92), host memory.
 * On success *out_kps (n records, sorted and de-duplicated exactly as
 * clean_keypoints, sift.cpp:20-24) is allocated by the library; release it
 * with sift_hip_free. If out_desc_f32 is non-null it receives n*128 floats:
 * the normalised descriptor h*norm_inv of convert_hist_to_desc
 * (sift.cpp:599-601) before the x512 quantisation (for the 1e-4 check).
 */
int sift_hip_detect(sift_ctx* ctx, const double* hwc, int w, int h, int c,
                    const sift_params* p, sift_kp** out_kps, size_t* out_n,
                    float** out_desc_f32);

/* Same, but `d_hwc` is a device pointer on the context's device (input
 * already resident in HBM). */
int sift_hip_detect_device(sift_ctx* ctx, const double* d_hwc, int w, int h,
                           int c, const sift_params* p, sift_kp** out_kps,
                           size_t* out_n, float** out_desc_f32);

void sift_hip_free(void* p);
const char* sift_hip_strerror(int status);

/* ---- jobs: batches of images, pipelined ------------------------------- */
/*
 * A job is 1..SIFT_MAX_BATCH images of the same w x h x c and parameters,
 * each processed exactly as detect_keypoints_and_descriptors would
 * (reference sift.cpp:712-776 is a pure function of one image); every kernel
 * of a job covers all its images in one launch. Up to SIFT_MAX_INFLIGHT jobs
 * can be in flight per context: submit job k+1 before waiting on job k and
 * the device works on k+1 while the host finalises k.
 *
 * Input kinds: the reference Image buffer (interleaved HWC doubles,
 * image_io.cpp:81-92) in host or device memory, or the 8-bit pixels stb
 * decodes (image_io.cpp:20-35; converted to double on the device, exactly).
 * Host double images whose values are all integers 0..255 (every
 * stb-decoded Image) are uploaded as bytes; the results are identical.
 * Device / host input buffers must stay valid until sift_hip_wait returns.
 * Pixel values must be finite (the reference's loader only produces 0..255):
 * host double images holding a NaN or an infinity are rejected with
 * SIFT_ERR_ARG; device double images are not scanned, and such values give
 * unspecified keypoints.
 */
#define SIFT_INPUT_F64_HOST 0
#define SIFT_INPUT_F64_DEVICE 1
#define SIFT_INPUT_U8_HOST 2
#define SIFT_INPUT_U8_DEVICE 3
#define SIFT_MAX_BATCH 16
#define SIFT_MAX_INFLIGHT 8

/* Enqueue a job; *ticket identifies it. SIFT_ERR_STATE when
 * SIFT_MAX_INFLIGHT jobs are already in flight (wait/fetch one first). */
int sift_hip_submit(sift_ctx* ctx, const void* const* images, int n_images, int input_kind,
                    int w, int h, int c, const sift_params* p, int want_desc_f32,
                    int* ticket);

/* Block until the job is finalised (sorted and de-duplicated per image, as
 * clean_keypoints, sift.cpp:20-24); counts[b] (n_images entries, optional)
 * = keypoints of image b, *total = their sum. */
int sift_hip_wait(sift_ctx* ctx, int ticket, size_t* counts, size_t* total);

/* Copy the job's keypoints into caller storage (total records, image-major:
 * image 0's sorted list, then image 1's, ...) and, if requested at submit,
 * total*128 normalised descriptor floats; releases the job. out == NULL
 * releases it without copying. Waits first if needed. */
int sift_hip_fetch(sift_ctx* ctx, int ticket, sift_kp* out, float* desc_f32);

/* Same as sift_hip_fetch, but the records go to DEVICE memory d_out (cap
 * records, on the context's device; image-major, identical bytes): gathered
 * on the device from the records the kernels left in HBM, only a 12-byte
 * (index, size) pair per keypoint crosses PCIe. Complete on return. Used by
 * the multi-GPU driver to feed the RCCL all-gather straight from HBM.
 * SIFT_ERR_ARG (job kept) when cap < the job's total. */
int sift_hip_fetch_device(sift_ctx* ctx, int ticket, void* d_out, size_t cap);

/* Asynchronous sift_hip_fetch_device: the device gather is enqueued on the
 * library's stream and `stream` (a hipStream_t of the caller, optional)
 * waits for it with an event, so the caller can hand d_out to a collective
 * with no host synchronisation. The job is released on return; its slot is
 * reused only once the gather has completed. With d_checksum (device
 * memory, optional) the wrapping 64-bit sum of every 8-byte word of the
 * records written is stored there (zeroed first), for
 * sift_hip_verify_slots. */
int sift_hip_fetch_device_async(sift_ctx* ctx, int ticket, void* d_out, size_t cap,
                                void* stream, uint64_t* d_checksum);

/* Exchange verification for the multi-GPU driver: n_slots slots of
 * slot_bytes each at d_slots (device memory); slot r holds at 8-byte word
 * count_word its record count n, at words [sum_word, sum_word + n_sum_words)
 * the sender's checksums of consecutive pieces of its records (one
 * sift_hip_fetch_device_async each), and the n 168-byte records after
 * hdr_rows header rows of 168 bytes. Every slot whose records' wrapping word
 * sum differs from the sum of its checksums (or whose n exceeds cap_rows)
 * adds 1 to *d_bad (device memory). Enqueued on `stream` (default: the
 * context's), no host wait. Calls of one context share its scratch and run
 * in call order on the device, whatever their streams (each waits for the
 * previous call's completion event). */
int sift_hip_verify_slots(sift_ctx* ctx, const void* d_slots, int n_slots, size_t slot_bytes,
                          int hdr_rows, int count_word, int sum_word, int n_sum_words,
                          size_t cap_rows, uint64_t* d_bad, void* stream);

/* ---- multi-GPU record exchange without torch ----- */
/*
 * A batch of images shards one image per GPU (rank r detects images
 * i % nranks == r; the reference function is pure per image,
 * src/sift.cpp:712-776). These give a C++ batch driver the one exchange:
 * every rank receives every image's final records, over RCCL (xGMI) in two
 * phases, since RCCL has no all-gather-v: the ranks' (image id, count)
 * tables, then the records padded to the largest rank's count (padding
 * dropped on the device). Same bytes as the torch path
 * (sift-project_amd/sift_dist.py allgather_records). RCCL is loaded on first
 * use (dlopen librccl.so.1); SIFT_ERR_NO_COMM when it is missing.
 *
 * Communicators: sift_hip_comm_init_all — one process drives every listed
 * device (ncclCommInitAll; comms[i] is rank i on devices[i]); then call
 * sift_hip_allgather_records for every rank concurrently, one host thread
 * per rank. Or one process per GPU: rank 0 gets an id with
 * sift_hip_comm_unique_id, shares it out of band, every rank calls
 * sift_hip_comm_init_rank.
 */
#define SIFT_COMM_ID_BYTES 128
typedef struct sift_comm sift_comm;
int sift_hip_comm_unique_id(unsigned char id[SIFT_COMM_ID_BYTES]);
int sift_hip_comm_init_rank(const unsigned char id[SIFT_COMM_ID_BYTES], int nranks, int rank,
                            int device, sift_comm** out);
int sift_hip_comm_init_all(int n_devices, const int* devices, sift_comm** comms);
int sift_hip_comm_destroy(sift_comm* comm);
int sift_hip_comm_rank(const sift_comm* comm, int* rank, int* nranks);

/* Collective over every rank of `comm` (each rank calls it once). max_local
 * is a collective argument like an all-gather's count: every rank passes the
 * same value (checked: a mismatch returns SIFT_ERR_ARG on every rank). This
 * rank's n_local (<= max_local) images: image ids[j] has counts[j] final
 * records, image-major in d_recs (device memory, e.g. from
 * sift_hip_fetch_device). On return every rank's d_out (device, cap_out
 * records) holds all ranks' records rank-major (rank 0's images in its
 * order, then rank 1's, ...), *n_out their total, and the host arrays
 * out_ids / out_counts (nranks * max_local entries, rank-major, id -1 for an
 * empty entry) describe them. Blocking (the host waits for the counts and
 * the final copies); `stream` optional. *n_out > cap_out: SIFT_ERR_ARG after
 * the collectives completed, nothing written to d_out.
 * No local failure leaves a peer blocked: a rank with a bad argument, or one
 * that cannot allocate or stage its payload, still enters every collective
 * of the call; the ranks agree on the failure before the payload moves, the
 * failing rank returns its own error and the others SIFT_ERR_PEER
 * (csrc/sift_exchange.h). */
int sift_hip_allgather_records(sift_comm* comm, const sift_kp* d_recs, const int64_t* ids,
                               const size_t* counts, int n_local, int max_local, sift_kp* d_out,
                               size_t cap_out, int64_t* out_ids, size_t* out_counts,
                               size_t* n_out, void* stream);

/* submit + wait + fetch into library-allocated storage (sift_hip_free):
 * *out_kps image-major, counts[b] per image. */
int sift_hip_detect_batch(sift_ctx* ctx, const void* const* images, int n_images,
                          int input_kind, int w, int h, int c, const sift_params* p,
                          sift_kp** out_kps, size_t* counts, float** out_desc_f32);

/* ---- matcher -------------------------------------------------------------- */
/*
 * Brute-force 2-NN ratio-test matcher (reference match_keypoints,
 * src/sift.cpp:783-815, with euclid_dist :688-695): for each record i1 of
 * kps1, the nearest (i2) and second-nearest records of kps2 by Euclidean
 * distance over the 128 descriptor bytes; a match when
 * best < ratio_threshold * second (second = DBL_MAX when n2 == 1). Matches
 * come in increasing i1 order, as the reference's vector; ties resolve as the
 * reference's scan (lowest i2 wins). n2 == 0 gives no matches (the reference
 * is undefined there for ratio > 1). *out is allocated by the library
 * (release with sift_hip_free; NULL when *n_out == 0).
 */
typedef struct sift_match_pair {
    uint32_t i1;      /* index into kps1 (KeypointMatch::kp1) */
    uint32_t i2;      /* index into kps2 (KeypointMatch::kp2) */
    double distance;  /* KeypointMatch::distance */
} sift_match_pair;

int sift_hip_match(sift_ctx* ctx, const sift_kp* kps1, size_t n1, const sift_kp* kps2,
                   size_t n2, double ratio_threshold, sift_match_pair** out, size_t* n_out);

/* Same with both record arrays resident on the context's device. */
int sift_hip_match_device(sift_ctx* ctx, const sift_kp* d_kps1, size_t n1,
                          const sift_kp* d_kps2, size_t n2, double ratio_threshold,
                          sift_match_pair** out, size_t* n_out);

/* ---- stitching consumer ------------------------------ */
/*
 * The reference's consumer of detect + match is its stitching notebook
 * (stitching/sift_stitch.ipynb, absent from the checkout: .MISSING_LARGE_BLOBS:3);
 * its inputs are the datasets' image sequences and their stitch graphs
 * (stitching/collection/Dataset/ * /<name>-STITCH-GRAPH.txt). These two entry
 * points are the data-parallel parts of a homography stitcher built on the
 * matcher above; sift-project_amd/sift_stitch.py drives them over a graph.
 *
 * RANSAC homography dst ~ H * src from n point pairs (x, y interleaved, e.g.
 * matched keypoint coordinates): hypothesis h draws 4 distinct pairs with a
 * splitmix64 stream seeded by (seed, h), solves the 8x8 DLT system with
 * h33 = 1 (Gaussian elimination, partial pivoting; singular pivot -> no
 * model), and counts the pairs whose squared reprojection error is below
 * threshold^2 — one wavefront per hypothesis on the device. The model with
 * the most inliers (ties: lowest h) is refitted refine_iters times by linear
 * least squares over its inliers (host, 8x8 normal equations), the inlier
 * set recounted after each refit. H is row-major, H[8] = 1. inliers (n
 * bytes, optional) gets the final inlier mask. SIFT_ERR_ARG when n < 4;
 * *n_inliers = 0 and H = identity when no hypothesis yields a model.
 */
typedef struct sift_ransac_params {
    int n_hyp;          /* hypotheses (default 4096, at most 1 << 20) */
    int refine_iters;   /* least-squares refits on the inliers (default 2) */
    double threshold;   /* inlier reprojection error, pixels (default 3.0) */
    uint64_t seed;      /* hypothesis sampler seed (default 0x5EED) */
} sift_ransac_params;

void sift_ransac_params_default(sift_ransac_params* p);

int sift_hip_ransac_homography(sift_ctx* ctx, const double* src_xy, const double* dst_xy,
                               size_t n, const sift_ransac_params* p, double* H,
                               unsigned char* inliers, size_t* n_inliers);

/* Inlier count of every hypothesis (n_hyp ints; -1 = no model), the device
 * scores behind sift_hip_ransac_homography (parity tests). */
int sift_hip_ransac_scores(sift_ctx* ctx, const double* src_xy, const double* dst_xy, size_t n,
                           const sift_ransac_params* p, int* scores);

/*
 * Panorama compositing: every canvas pixel (X, Y) of out (out_w x out_h x c
 * bytes, host) is the feather-weighted mean of the images that cover it:
 * image i (w[i] x h[i] x c bytes, host, HWC) is sampled bilinearly (clamped
 * neighbours) at (x, y) = Hinv_i * (X, Y, 1) (Hinv: 9 doubles per image,
 * row-major, image-from-canvas) when 0 <= x <= w-1 and 0 <= y <= h-1, with
 * weight min(x + 1, w - x, y + 1, h - y); out = floor(sum / weight + 0.5),
 * 0 where nothing covers it. Images are accumulated in index order.
 */
int sift_hip_warp_blend(sift_ctx* ctx, const unsigned char* const* images, const int* w,
                        const int* h, int c, int n_images, const double* Hinv, int out_w,
                        int out_h, unsigned char* out);

/* ---- introspection of the last finalised job (tests, bench, multi-GPU) -- */
/* (valid until a later submit reuses that job's slot; counts sum over the
 * job's images) */

/* Pipeline counts of the last detect: extrema candidates, refined
 * keypoints, oriented keypoints (pre-dedup), final keypoints, octaves. */
typedef struct sift_counts {
    int64_t extrema;
    int64_t refined;
    int64_t oriented;
    int64_t final_n;
    int octaves;
    int levels_per_octave;
    int octave0_w;
    int octave0_h;
} sift_counts;
int sift_hip_last_counts(sift_ctx* ctx, sift_counts* out);

/* Copy Gaussian level G[octave][level] of the last detect to host
 * (w_o*h_o doubles, row-major). Level 0 of octave o>0 is the decimated base. */
int sift_hip_copy_level(sift_ctx* ctx, int octave, int level, double* host_out,
                        size_t cap_elems, int* w_out, int* h_out);

/* Copy the extrema candidate list of the last detect (unordered). */
int sift_hip_copy_extrema(sift_ctx* ctx, sift_extremum* host_out,
                          size_t cap, size_t* n_out);

/* Device-side pre-dedup keypoint records of the last detect (n records of
 * sift_kp, unordered): copied device-to-device into `d_dst` (a buffer on the
 * same device), then synchronised. NOTE: these are the kernels' records
 * before clean_keypoints, and their size field is the device's (ocml pow),
 * not the final glibc-exact size; sift_hip_fetch_device gives the final,
 * sorted, de-duplicated records with exact sizes. */
int sift_hip_copy_records_device(sift_ctx* ctx, void* d_dst, size_t cap,
                                 size_t* n_out);

/* Host-side wall time (ms) of the phases of the last detect: [0] plan +
 * enqueue of every kernel, [1] wait for the device pipeline, [2] download of
 * the keypoint records, [3] final size + clean_keypoints, [4] output
 * assembly, [5] the part of [1]-[3] the host spent blocked on device
 * events (the rest is host work: per-chain sizes and sorted runs, merge).
 * Writes min(n, 6) values. */
int sift_hip_last_timing(sift_ctx* ctx, double* ms, int n);

/* The context's HIP stream (hipStream_t), for event timing. */
void* sift_hip_stream(sift_ctx* ctx);

/*
 * Per-kernel timing of the pyramid (blur) kernels with HIP events on the
 * context stream. When enabled, every blur launch is bracketed by events;
 * sift_hip_blur_profile returns the accumulated kernel time (ms), the
 * number of launches and their algorithmic HBM bytes (read src once, write
 * dst once: 16 B/px, plus 8 B per decimated px) since the last reset.
 */
int sift_hip_set_profiling(sift_ctx* ctx, int enable);
int sift_hip_blur_profile(sift_ctx* ctx, double* ms, int64_t* launches,
                          double* bytes, int reset);

/* The same per row: SIFT_PROF_PYRAMID + o = pyramid launches of octave o
 * (the LDS-resident small-octave launch counts under its first octave),
 * SIFT_PROF_EXTREMA = extrema launches (algorithmic bytes: every Gaussian
 * level read once per pixel), SIFT_PROF_REFINE / _ORIENT / _DESC = the
 * keypoint stages' launches (bytes 0). Each array holds SIFT_PROF_ROWS
 * entries. */
#define SIFT_PROF_PYRAMID 0
#define SIFT_PROF_EXTREMA 16
#define SIFT_PROF_REFINE 17
#define SIFT_PROF_ORIENT 18
#define SIFT_PROF_DESC 19
#define SIFT_PROF_ROWS 20
int sift_hip_profile_table(sift_ctx* ctx, double* ms, double* bytes, int64_t* launches,
                           int reset);

/* ---- synthetic input (bench + tests) ----------------------------------- */
/*
 * Deterministic synthetic gray image, bit-reproducible on any IEEE-754
 * machine (integer RNG + basic-op polynomials, no libm): background
 * 128+40*sin(x/37)*cos(y/53) plus `nblobs` Gaussian blobs with
 * sigma in [1.5, 1.5+smax] and amplitude in [-100,100], clamped to [0,255]
 * and rounded to integers (SURVEY §6 workload class, portable generator).
 * out: w*h doubles. channels==3 replicates a tinted RGB version.
 */
int sift_synth_image(int w, int h, int channels, int64_t nblobs, double smax,
                     uint64_t seed, double* out);

#ifdef __cplusplus
}
#endif

#endif /* SIFT_HIP_H */
