/* orbx_match.h — C ABI of the descriptor matchers (replaces ORB_SLAM2::ORBmatcher).
 *
 * The reference class is include/ORBmatcher.h:37-128 / src/ORBmatcher.cc.  Its methods read
 * Frame / KeyFrame / MapPoint objects; this boundary takes the plain arrays those objects
 * hold instead, so a thin C++ facade can keep the reference signatures:
 *
 *   orbx_featureset  = the per-frame arrays a matcher reads: mvKeysUn, mDescriptors,
 *                      mvuRight, mFeatVec (DBoW2::FeatureVector, as CSR) and mGrid (as CSR).
 *   "valid" / "has_mp" / "claimed" masks = the MapPoint* arrays reduced to the one bit each
 *                      method tests (non-NULL and !isBad(), Observations()>0, ...).
 *   orbx_proj_query  = the projection of one MapPoint (u, v, ur, radius, levels), computed by
 *                      the caller with the reference's own cv::Mat code, as SURVEY §8(b) puts
 *                      the boundary; the window search, Hamming distances, greedy claims and
 *                      rotation-consistency filter run on the GPU.
 *
 * Outputs are feature indices (-1 = no match); the facade turns them back into MapPoint*.
 * Every function returns the reference method's return value in *nmatches.  All host-pointer
 * entry points copy their inputs to the device, run on the matcher's stream and wait.
 * Functions named *_device take device pointers and run on the caller's stream.
 *
 * A matcher handle is not re-entrant (its device workspace is reused); use one per thread,
 * as the reference's Tracking / LocalMapping / LoopClosing threads each own their ORBmatcher.
 */
#ifndef ORBX_MATCH_H
#define ORBX_MATCH_H

#include "orbx.h"

#ifdef __cplusplus
extern "C" {
#endif

/* src/ORBmatcher.cc:37-39 */
enum { ORBX_TH_HIGH = 100, ORBX_TH_LOW = 50, ORBX_HISTO_LENGTH = 30 };

/* One Frame or KeyFrame as seen by the matchers.  Feature i has keys[i] (mvKeysUn: pt,
 * octave and angle are read), desc + 32*i (mDescriptors row i) and u_right[i] (mvuRight;
 * NULL = every feature monocular, i.e. -1).
 * FeatureVector (Thirdparty/DBoW2/DBoW2/FeatureVector.h): node j has id node_id[j] (strictly
 * ascending, the std::map order) and features node_feat[node_off[j] .. node_off[j+1]) in the
 * order DBoW2 pushed them; every feature index appears in at most one node (transform()
 * adds each feature to exactly one node, FeatureVector.cpp:31-45).
 * Grid (Frame::mGrid / KeyFrame::mGrid): cell (ix, iy) = grid_feat[grid_off[c] ..
 * grid_off[c+1]) with c = ix*grid_rows + iy, indices in AssignFeaturesToGrid order
 * (Frame.cc:243-258); min_x/min_y/max_x/max_y = mnMinX.., grid_inv_w/h =
 * mfGridElementWidthInv / mfGridElementHeightInv.  Grid fields are only read by the
 * projection searches and may be zero/NULL elsewhere. */
typedef struct {
    int32_t n;
    const orbx_keypoint* keys;
    const uint8_t* desc;
    const float* u_right;
    int32_t n_nodes;
    const uint32_t* node_id;
    const int32_t* node_off;
    const int32_t* node_feat;
    int32_t grid_cols, grid_rows;
    const int32_t* grid_off;
    const int32_t* grid_feat;
    float min_x, min_y, max_x, max_y;
    float grid_inv_w, grid_inv_h;
} orbx_featureset;

typedef struct {
    float nnratio;              /* ORBmatcher(nnratio, ...) default 0.6       */
    int32_t check_orientation;  /* ORBmatcher(..., checkOri) default true     */
    int32_t device;             /* HIP device ordinal                         */
} orbx_matcher_params;

typedef struct orbx_matcher orbx_matcher;

/* ORBmatcher::ORBmatcher (src/ORBmatcher.cc:41-43). */
orbx_status orbx_matcher_create(const orbx_matcher_params* params, orbx_matcher** out);
orbx_status orbx_matcher_destroy(orbx_matcher* m);

/* ORBmatcher::ComputeThreeMaxima (src/ORBmatcher.cc:1669-1710) on bin counts histo[L]
 * (host, no device work). */
void orbx_compute_three_maxima(const int32_t* histo, int32_t L, int32_t* ind1, int32_t* ind2,
                               int32_t* ind3);

/* ORBmatcher::SearchByBoW(KeyFrame*, Frame&, vector<MapPoint*>&) (src/ORBmatcher.cc:182-319).
 * kf_valid[i] = pKF->GetMapPointMatches()[i] && !isBad().  match_f[n_f]: for each frame
 * feature, the keyframe feature whose MapPoint it received (vpMapPointMatches), or -1. */
orbx_status orbx_search_by_bow_kf_frame(orbx_matcher* m, const orbx_featureset* kf,
                                        const uint8_t* kf_valid, const orbx_featureset* f,
                                        int32_t* match_f, int32_t* nmatches);

/* ORBmatcher::SearchByBoW(KeyFrame*, KeyFrame*, vector<MapPoint*>&) (:563-696).
 * valid1/valid2 as above; match12[n1] = KF2 feature matched to each KF1 feature or -1. */
orbx_status orbx_search_by_bow_kf_kf(orbx_matcher* m, const orbx_featureset* kf1,
                                     const uint8_t* valid1, const orbx_featureset* kf2,
                                     const uint8_t* valid2, int32_t* match12, int32_t* nmatches);

/* ORBmatcher::SearchForTriangulation (:702-872) + CheckDistEpipolarLine (:147-167).
 * has_mp1/has_mp2[i] = GetMapPoint(i) != NULL.  F12: row-major 3x3 (F12.at<float>(r,c) =
 * F12[3r+c]).  (ex, ey): the epipole the reference computes at :709-715.  sigma2_2 /
 * scale_2: pKF2->mvLevelSigma2 / mvScaleFactors (nlevels).  pairs: (idx1, idx2) in idx1
 * order, up to pair_cap pairs (ORBX_ERR_CAPACITY if more; *nmatches = the count). */
orbx_status orbx_search_for_triangulation(orbx_matcher* m, const orbx_featureset* kf1,
                                          const uint8_t* has_mp1, const orbx_featureset* kf2,
                                          const uint8_t* has_mp2, const float* F12, float ex,
                                          float ey, const float* sigma2_2,
                                          const float* scale_2, int32_t nlevels,
                                          int32_t only_stereo, int32_t* pairs,
                                          int32_t pair_cap, int32_t* nmatches);

/* Projection searches: one query per MapPoint, in the reference's MapPoint order (the
 * greedy claims follow it).  u, v, radius: the GetFeaturesInArea arguments; ur: projected
 * right-image x (mTrackProjXR at :96, u - mbf*invzc at :1477, u - bf*invz at :924);
 * min_level/max_level: Frame::GetFeaturesInArea level arguments (-1 = unused, Frame.cc:373);
 * pred_level: the predicted octave for the matcher-side octave filters; angle: the source
 * keypoint angle for the rotation check (LastFrame / KeyFrame variants).  A query with
 * radius < 0 is inactive (no search, result -1). */
typedef struct {
    float u, v, ur, radius;
    int32_t min_level, max_level, pred_level;
    float angle;
} orbx_proj_query;

typedef enum {
    /* SearchByProjection(Frame&, vector<MapPoint*>, th)   :46-132  (Frame grid + levels,
       skip claimed, stereo check, best+2nd with levels, TH_HIGH, ratio if same level) */
    ORBX_PROJ_FRAME_MAPPOINTS = 0,
    /* SearchByProjection(KeyFrame*, Scw, vpPoints, vpMatched, th)  :321-434 (KeyFrame grid,
       skip claimed, octave in [pred-1, pred], TH_LOW) */
    ORBX_PROJ_KF_SCW = 1,
    /* SearchByProjection(Frame&, const Frame& LastFrame, th, bMono) :1392-1538 (Frame grid +
       levels, skip claimed, stereo check, TH_HIGH, rotation check) */
    ORBX_PROJ_LAST_FRAME = 2,
    /* SearchByProjection(Frame&, KeyFrame*, sAlreadyFound, th, ORBdist) :1540-1667 (Frame
       grid + levels, skip claimed, ORBdist, rotation check) */
    ORBX_PROJ_KEYFRAME = 3,
    /* Fuse(KeyFrame*, vpMapPoints, th) :879-1029 (KeyFrame grid, octave filter, reprojection
       chi2 test, TH_LOW; no claims: the caller applies Replace/AddMapPoint in query order) */
    ORBX_PROJ_FUSE = 4,
    /* Fuse(KeyFrame*, Scw, vpPoints, th, vpReplacePoint) :1033-1156 (TH_LOW, no claims) */
    ORBX_PROJ_FUSE_SCW = 5,
    /* one direction of SearchBySim3 :1204-1281 / :1284-1361 (TH_HIGH, no claims) */
    ORBX_PROJ_SIM3 = 6,
    ORBX_PROJ_MODE_COUNT = 7
} orbx_proj_mode;

/* Runs one projection search of `mode` against `target`.  qdesc: nq x 32 query (MapPoint)
 * descriptors.  claimed[target->n] (may be NULL = none): features the search must skip from
 * the start (F.mvpMapPoints[i] with Observations()>0 for FRAME_MAPPOINTS / LAST_FRAME,
 * non-NULL for KEYFRAME, vpMatched[i] non-NULL for KF_SCW); ignored by FUSE/FUSE_SCW/SIM3.
 * inv_sigma2: target mvInvLevelSigma2 (FUSE only, may be NULL otherwise); nlevels its size.
 * orb_dist: the ORBdist argument (KEYFRAME only).  match_q[nq]: target feature matched to
 * each query, or -1, after the rotation-consistency filter where the mode has one. */
orbx_status orbx_search_by_projection(orbx_matcher* m, int32_t mode,
                                      const orbx_featureset* target, const uint8_t* claimed,
                                      const uint8_t* qdesc, const orbx_proj_query* q,
                                      int32_t nq, const float* inv_sigma2, int32_t nlevels,
                                      int32_t orb_dist, int32_t* match_q, int32_t* nmatches);

/* orbx_search_by_projection with per-query flags and call flags.
 * qflags[nq] (may be NULL = all 0): ORBX_QF_NO_CLAIM marks a query whose MapPoint has no
 * observations (Observations() == 0, e.g. the stereo "temporal" points Tracking::UpdateLastFrame
 * puts into the last frame).  The reference's skip test for an already matched feature is
 * F.mvpMapPoints[i] && F.mvpMapPoints[i]->Observations() > 0 (:90-92, :1471-1473), so such a
 * query's match does not keep later queries off its feature (a later match overwrites it).
 * Only the FRAME_MAPPOINTS and LAST_FRAME modes read the flag.
 * flags: ORBX_PROJ_PREFILTER returns every accepted query's feature without the
 * rotation-consistency filter (LAST_FRAME / KEYFRAME), *nmatches = the accepted count, so the
 * caller can apply the reference's per-feature filter itself (rotHist holds feature indices,
 * :1508 / :1637: with overwritten matches a feature can sit in two bins).  LAST_FRAME with
 * check_orientation and any ORBX_QF_NO_CLAIM query requires ORBX_PROJ_PREFILTER
 * (ORBX_ERR_INVALID otherwise): the reference clears per feature (:1516-1535), which a
 * per-query filter cannot reproduce once a feature is matched twice.
 * Replaces the same ORBmatcher methods as orbx_search_by_projection, which equals this call
 * with qflags = NULL and flags = 0. */
enum { ORBX_QF_NO_CLAIM = 1 };
enum { ORBX_PROJ_PREFILTER = 1 };
orbx_status orbx_search_by_projection_ex(orbx_matcher* m, int32_t mode,
                                         const orbx_featureset* target, const uint8_t* claimed,
                                         const uint8_t* qdesc, const orbx_proj_query* q,
                                         const uint8_t* qflags, int32_t nq,
                                         const float* inv_sigma2, int32_t nlevels,
                                         int32_t orb_dist, int32_t flags, int32_t* match_q,
                                         int32_t* nmatches);

/* ORBmatcher::SearchBySim3 (:1158-1382).  q12[n1]: KF1 feature i's MapPoint projected into
 * KF2 (radius < 0 when the reference skips i1: no MapPoint, already matched, bad, or failed
 * the depth/image/distance tests); qdesc1: n1 x 32 MapPoint descriptors.  q21[n2] likewise
 * for KF2's MapPoints projected into KF1.  match12[n1] = idx2 where both directions agree
 * (vpMatches12[i1] = vpMapPoints2[idx2]), else -1; *nmatches = nFound. */
orbx_status orbx_search_by_sim3(orbx_matcher* m, const orbx_featureset* kf1,
                                const orbx_featureset* kf2, const uint8_t* qdesc1,
                                const orbx_proj_query* q12, int32_t n1, const uint8_t* qdesc2,
                                const orbx_proj_query* q21, int32_t n2, int32_t* match12,
                                int32_t* nmatches);

/* ORBmatcher::SearchForInitialization (:446-561).  prev_matched: n1 x 2 floats
 * (vbPrevMatched), updated in place for matched features like the reference (:555-558).
 * match12[n1] = vnMatches12. */
orbx_status orbx_search_for_initialization(orbx_matcher* m, const orbx_featureset* f1,
                                           const orbx_featureset* f2, float* prev_matched,
                                           int32_t window_size, int32_t* match12,
                                           int32_t* nmatches);

/* ---- batched, device-resident API (relocalisation / loop closure / local mapping) -------
 * A keyframe database: nkf featuresets concatenated.  Keyframe k owns features
 * [feat_off[k], feat_off[k+1]) of keys/desc/u_right/flag (feature indices inside a keyframe
 * are local, 0-based) and FeatureVector nodes [node_off[k], node_off[k+1]) of node_id /
 * node_feat_off (absolute offsets into node_feat, which holds local feature indices;
 * node_feat_off has node_off[nkf] + 1 entries).  flag[i]: MapPoint mask (valid for BoW,
 * has_mp for triangulation).  All pointers are device memory. */
typedef struct {
    int32_t nkf;
    int32_t max_feat;              /* host-known bound on any keyframe's feature count
                                      (sizes the on-chip workspace); a keyframe above it
                                      is skipped (outputs -1, count 0) and flagged for
                                      orbx_matcher_sync */
    const int32_t* feat_off;
    const orbx_keypoint* keys;
    const uint8_t* desc;
    const float* u_right;          /* may be NULL (all monocular) */
    const uint8_t* flag;
    const int32_t* node_off;
    const uint32_t* node_id;
    const int32_t* node_feat_off;
    const int32_t* node_feat;
    /* Optional (all NULL, or all set by orbx_kf_db_node_order): the features again in node
     * order, entry p = keyframe-local feature node_feat[p] of p's keyframe.  A per-node matcher
     * (SearchForTriangulation) then reads each node's keys, descriptors, stereo and flag as
     * contiguous runs instead of one gather per feature (each gather a cache line of its own:
     * 4.3x the bytes it uses).  node_desc 16-byte aligned; node_u_right NULL iff u_right is. */
    const orbx_keypoint* node_keys;
    const uint8_t* node_desc;
    const float* node_u_right;
    const uint8_t* node_flag;
} orbx_kf_db;

/* Fills a database's node-order copies (orbx_kf_db node_keys / node_desc / node_u_right /
 * node_flag): device arrays of n = db->node_feat_off[db->node_off[db->nkf]] entries each
 * (d_u_right may be NULL when db->u_right is), on `stream`; the caller then points the
 * database's node_* fields at them.  A database whose flags change (MapPoints added) must be
 * reordered again. */
orbx_status orbx_kf_db_node_order(orbx_matcher* m, const orbx_kf_db* db, int32_t n,
                                  orbx_keypoint* d_keys, uint8_t* d_desc, float* d_u_right,
                                  uint8_t* d_flag, void* stream);

/* SearchByBoW(KeyFrame*, Frame&) of every keyframe of `db` against one frame `f` (device
 * featureset; grid unused) — the relocalisation candidate loop of Tracking.cc:1479-1500.
 * d_match: device [db->nkf][f->n] (KF-local feature index per frame feature, or -1);
 * d_nmatches: device [db->nkf]. */
orbx_status orbx_search_by_bow_kf_frame_batch_device(orbx_matcher* m, const orbx_kf_db* db,
                                                     const orbx_featureset* f,
                                                     int32_t* d_match, int32_t* d_nmatches,
                                                     void* stream);

/* SearchForTriangulation over njobs keyframe pairs (kf1[j], kf2[j]) of `db` (the
 * LocalMapping::CreateNewMapPoints loop, LocalMapping.cc:271-276).  d_F12: device njobs x 9,
 * d_epi: device njobs x 2 (ex, ey); sigma2 / scale: HOST tables of nlevels floats shared by
 * all keyframes.  d_match12: device, one slot per KF1 feature of each job laid out at
 * d_job_off[j] (device, njobs+1, = prefix of KF1 sizes); d_nmatches: device [njobs]. */
orbx_status orbx_search_for_triangulation_batch_device(
    orbx_matcher* m, const orbx_kf_db* db, int32_t njobs, const int32_t* d_kf1,
    const int32_t* d_kf2, const float* d_F12, const float* d_epi, const float* sigma2,
    const float* scale, int32_t nlevels, int32_t only_stereo, const int32_t* d_job_off,
    int32_t* d_match12, int32_t* d_nmatches, void* stream);

/* SearchByProjection over njobs frames at once — one Tracking::SearchLocalPoints
 * (Tracking.cc:1297-1347, ORBmatcher.cc:41-136) per frame, or any other
 * non-initialisation orbx_proj_mode, each job independent of the others.
 * `frames` holds DEVICE pointers to the concatenation of the frames: keys / desc / u_right
 * (u_right may be NULL) with frame j's features at [d_feat_off[j], d_feat_off[j+1]);
 * grid_off = njobs blocks of grid_cols*grid_rows+1 entries (frame-local positions, frame j's
 * block at j*(cells+1)); grid_feat with frame j's entries from d_grid_off[j] (frame-local
 * feature indices).  Grid geometry (cols, rows, bounds, inverse cell sizes) is shared: one
 * camera.  frames->n is ignored; max_feat (host) bounds every frame's size.
 * Queries: d_qdesc / d_q with frame j's at [d_q_off[j], d_q_off[j+1]), nq in total.
 * d_claimed: device, one byte per feature of the concatenation (already-matched features of
 * the KEYFRAME / FUSE modes), or NULL.  inv_sigma2: HOST table of nlevels floats.
 * Outputs (device): d_match[nq] frame-local feature index or -1, d_nmatches[njobs].
 * Scratch belongs to the matcher: calls on one matcher must share `stream` or be serialised.
 * A frame above max_feat gets no matches and is flagged for orbx_matcher_sync. */
orbx_status orbx_search_by_projection_batch_device(
    orbx_matcher* m, int32_t mode, const orbx_featureset* frames, int32_t njobs,
    const int32_t* d_feat_off, const int32_t* d_grid_off, int32_t max_feat,
    const uint8_t* d_claimed, const uint8_t* d_qdesc, const orbx_proj_query* d_q,
    const int32_t* d_q_off, int32_t nq, const float* inv_sigma2, int32_t nlevels,
    int32_t orb_dist, int32_t* d_match, int32_t* d_nmatches, void* stream);

/* Brute-force Hamming top-2 of nq query descriptors (q: nq x 32) against ndb database rows
 * (db: ndb x 32) — SURVEY §8(b) orbx_hamming_bf_top2 / §8(e) C4.  The semantics are the best /
 * second loop of the ORBmatcher searches (src/ORBmatcher.cc:232-256) run over every row in
 * order: bestDist1 = bestDist2 = 256 initially, `dist < bestDist1` moves the best to the
 * second, else `dist < bestDist2` updates the second.  best_idx[i] = the first row at the least
 * distance (-1 if no row is below 256), best_dist[i] that distance (256 if none),
 * second_dist[i] the second least distance (equal to best_dist[i] on a tie, 256 if none).
 * Host pointers; the database is copied to the device for the call (keep a large database
 * resident and use the _device form instead). */
orbx_status orbx_hamming_bf_top2(orbx_matcher* m, const uint8_t* q, int32_t nq,
                                 const uint8_t* db, int64_t ndb, int32_t* best_idx,
                                 int32_t* best_dist, int32_t* second_dist);
/* The same on device arrays, on the caller's stream; best_idx is offset by idx_base (a shard
 * of a larger database reports global row numbers, so per-shard results merge in shard order
 * with distributed.merge_top2).  ndb < 2^31 - idx_base.  The partial results live in the
 * matcher's scratch: a call on another stream than the previous call's waits (on the device,
 * by an event) until that call's kernels are done with it. */
orbx_status orbx_hamming_bf_top2_device(orbx_matcher* m, const uint8_t* d_q, int32_t nq,
                                        const uint8_t* d_db, int64_t ndb, int64_t idx_base,
                                        int32_t* d_best_idx, int32_t* d_best_dist,
                                        int32_t* d_second_dist, void* stream);

/* The kernel the brute-force top-2 of a matcher runs its distances in (results are identical):
 * ORBX_BF_MFMA (the default): k_bf_mfma, +-1 int8 dot products on the matrix cores;
 * ORBX_BF_VALU: k_bf_top2, v_xor + v_bcnt on the vector ALUs (north_star's "no MFMA" form). */
enum { ORBX_BF_MFMA = 0, ORBX_BF_VALU = 1 };
orbx_status orbx_matcher_set_bf_kernel(orbx_matcher* m, int32_t kernel);
/* The kernel name of that choice ("k_bf_mfma" / "k_bf_top2"); NULL for an unknown value. */
const char* orbx_bf_kernel_name(int32_t kernel);
/* The default's name ("k_bf_mfma"). */
const char* orbx_bf_kernel(void);

/* Waits for `stream` and returns ORBX_ERR_CAPACITY if a batched call on this matcher met a
 * keyframe above max_feat since the last sync (the flag is then cleared). */
orbx_status orbx_matcher_sync(orbx_matcher* m, void* stream);

/* MapPoint::ComputeDistinctiveDescriptors (src/MapPoint.cc:252-313) for npoints map points:
 * point p's observed descriptors are rows [off[p], off[p+1]) of desc (n x 32, in the order
 * the reference walks mObservations, skipping bad keyframes).  best[p] = the row (relative
 * to off[p]) with the least median distance to the others (first on ties), or -1 when the
 * point has no descriptor (the reference then keeps mDescriptor).  At most
 * ORBX_MAX_OBSERVATIONS rows per point (ORBX_ERR_UNSUPPORTED above). */
enum { ORBX_MAX_OBSERVATIONS = 256 };
orbx_status orbx_compute_distinctive_descriptors(orbx_matcher* m, const uint8_t* desc,
                                                 const int32_t* off, int32_t npoints,
                                                 int32_t* best);
/* Same on device arrays, on the caller's stream (points above the limit get -1 and are
 * flagged for orbx_matcher_sync). */
orbx_status orbx_compute_distinctive_descriptors_device(orbx_matcher* m, const uint8_t* d_desc,
                                                        const int32_t* d_off, int32_t npoints,
                                                        int32_t* d_best, void* stream);

/* ---- per-kernel timing for the matcher handle ------------------------------------------ */
typedef enum {
    ORBX_MK_BOW = 0, ORBX_MK_TRIANGULATE, ORBX_MK_PROJ_SEARCH, ORBX_MK_PROJ_RESOLVE,
    ORBX_MK_DISTINCTIVE, ORBX_MK_BF, ORBX_MK_COUNT
} orbx_match_kernel_id;
orbx_status orbx_matcher_profile_enable(orbx_matcher* m, int on);
orbx_status orbx_matcher_profile_collect(orbx_matcher* m, double* total_ms, int64_t* launches);
const char* orbx_match_kernel_name(int id);

#ifdef __cplusplus
}
#endif
#endif /* ORBX_MATCH_H */
