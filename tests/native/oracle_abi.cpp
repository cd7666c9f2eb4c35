// oracle_abi.cpp — TEST DOUBLE of the liborbx matcher entry points that integration/ORBmatcher.h
// calls, implemented by the query-level CPU oracle (oracle/orb_matcher_oracle.cpp).  It is linked
// only into tests/native/matcher_test_cpu (my_orb_slam2_amd/build.py build_matcher_test), so the
// CPU test suite can run the drop-in facade's host-side preparation and write-back (the cv::Mat
// projections, skip tests, claims, rotation histograms, Replace / AddObservation) against the
// object-level restatement (oracle/orb_matcher_objects.h) without a GPU.  It is never part of
// liborbx or of any product build: the GPU test runs the same program linked against liborbx.
#include <cstdint>
#include <cstring>
#include <vector>

#include "orbx_match.h"

extern "C" {
// oracle/orb_matcher_oracle.cpp
int oracle_descriptor_distance_m(const uint8_t* a, const uint8_t* b);
void oracle_three_maxima(const int32_t* counts, int L, int32_t* out3);
int oracle_search_by_bow_kf_frame(const orbx_featureset* KF, const uint8_t* valid,
                                  const orbx_featureset* F, float nnratio, int checkOri,
                                  int32_t* match);
int oracle_search_by_bow_kf_kf(const orbx_featureset* K1, const uint8_t* valid1,
                               const orbx_featureset* K2, const uint8_t* valid2, float nnratio,
                               int checkOri, int32_t* match12);
int oracle_search_for_triangulation(const orbx_featureset* K1, const uint8_t* has_mp1,
                                    const orbx_featureset* K2, const uint8_t* has_mp2,
                                    const float* F12, float ex, float ey, const float* sigma2,
                                    const float* scale, int onlyStereo, int checkOri,
                                    int32_t* match12);
int oracle_search_by_projection_ex(int mode, const orbx_featureset* T, const uint8_t* claimed_in,
                                   const uint8_t* qdesc, const orbx_proj_query* Q,
                                   const uint8_t* qflags, int nq, const float* inv_sigma2,
                                   int orb_dist, float nnratio, int checkOri, int prefilter,
                                   int32_t* match_q);
int oracle_search_by_sim3(const orbx_featureset* K1, const orbx_featureset* K2,
                          const uint8_t* qdesc1, const orbx_proj_query* q12, int n1,
                          const uint8_t* qdesc2, const orbx_proj_query* q21, int n2,
                          int32_t* match12);
int oracle_search_for_initialization(const orbx_featureset* F1, const orbx_featureset* F2,
                                     float* prev_matched, int windowSize, float nnratio,
                                     int checkOri, int32_t* vnMatches12);
}

struct orbx_matcher {
    orbx_matcher_params prm;
};

extern "C" {

const char* orbx_last_error(void) { return "oracle_abi test double"; }

int orbx_descriptor_distance(const uint8_t* a, const uint8_t* b) {
    return oracle_descriptor_distance_m(a, b);
}

void orbx_compute_three_maxima(const int32_t* histo, int32_t L, int32_t* ind1, int32_t* ind2,
                               int32_t* ind3) {
    int32_t o[3];
    oracle_three_maxima(histo, L, o);
    *ind1 = o[0];
    *ind2 = o[1];
    *ind3 = o[2];
}

orbx_status orbx_matcher_create(const orbx_matcher_params* params, orbx_matcher** out) {
    *out = new orbx_matcher{*params};
    return ORBX_OK;
}

orbx_status orbx_matcher_destroy(orbx_matcher* m) {
    delete m;
    return ORBX_OK;
}

orbx_status orbx_search_by_bow_kf_frame(orbx_matcher* m, const orbx_featureset* kf,
                                        const uint8_t* kf_valid, const orbx_featureset* f,
                                        int32_t* match_f, int32_t* nmatches) {
    *nmatches = oracle_search_by_bow_kf_frame(kf, kf_valid, f, m->prm.nnratio,
                                              m->prm.check_orientation, match_f);
    return ORBX_OK;
}

orbx_status orbx_search_by_bow_kf_kf(orbx_matcher* m, const orbx_featureset* kf1,
                                     const uint8_t* valid1, const orbx_featureset* kf2,
                                     const uint8_t* valid2, int32_t* match12, int32_t* nmatches) {
    *nmatches = oracle_search_by_bow_kf_kf(kf1, valid1, kf2, valid2, m->prm.nnratio,
                                           m->prm.check_orientation, match12);
    return ORBX_OK;
}

orbx_status orbx_search_for_triangulation(orbx_matcher* m, const orbx_featureset* kf1,
                                          const uint8_t* has_mp1, const orbx_featureset* kf2,
                                          const uint8_t* has_mp2, const float* F12, float ex,
                                          float ey, const float* sigma2_2, const float* scale_2,
                                          int32_t /*nlevels*/, int32_t only_stereo,
                                          int32_t* pairs, int32_t pair_cap, int32_t* nmatches) {
    std::vector<int32_t> m12((size_t)kf1->n + 1);
    *nmatches = oracle_search_for_triangulation(kf1, has_mp1, kf2, has_mp2, F12, ex, ey, sigma2_2,
                                                scale_2, only_stereo, m->prm.check_orientation,
                                                m12.data());
    int np = 0;
    for (int i = 0; i < kf1->n; ++i)
        if (m12[(size_t)i] >= 0) {
            if (np >= pair_cap) return ORBX_ERR_CAPACITY;
            pairs[2 * np] = i;
            pairs[2 * np + 1] = m12[(size_t)i];
            ++np;
        }
    return ORBX_OK;
}

orbx_status orbx_search_by_projection_ex(orbx_matcher* m, int32_t mode,
                                         const orbx_featureset* target, const uint8_t* claimed,
                                         const uint8_t* qdesc, const orbx_proj_query* q,
                                         const uint8_t* qflags, int32_t nq,
                                         const float* inv_sigma2, int32_t /*nlevels*/,
                                         int32_t orb_dist, int32_t flags, int32_t* match_q,
                                         int32_t* nmatches) {
    *nmatches = oracle_search_by_projection_ex(mode, target, claimed, qdesc, q, qflags, nq,
                                               inv_sigma2, orb_dist, m->prm.nnratio,
                                               m->prm.check_orientation,
                                               (flags & ORBX_PROJ_PREFILTER) != 0, match_q);
    return *nmatches < 0 ? ORBX_ERR_INVALID : ORBX_OK;
}

orbx_status orbx_search_by_sim3(orbx_matcher* /*m*/, const orbx_featureset* kf1,
                                const orbx_featureset* kf2, const uint8_t* qdesc1,
                                const orbx_proj_query* q12, int32_t n1, const uint8_t* qdesc2,
                                const orbx_proj_query* q21, int32_t n2, int32_t* match12,
                                int32_t* nmatches) {
    *nmatches = oracle_search_by_sim3(kf1, kf2, qdesc1, q12, n1, qdesc2, q21, n2, match12);
    return ORBX_OK;
}

orbx_status orbx_search_for_initialization(orbx_matcher* m, const orbx_featureset* f1,
                                           const orbx_featureset* f2, float* prev_matched,
                                           int32_t window_size, int32_t* match12,
                                           int32_t* nmatches) {
    *nmatches = oracle_search_for_initialization(f1, f2, prev_matched, window_size,
                                                 m->prm.nnratio, m->prm.check_orientation, match12);
    return ORBX_OK;
}

}  // extern "C"
