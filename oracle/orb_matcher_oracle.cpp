// orb_matcher_oracle.cpp — CPU restatement of src/ORBmatcher.cc (TEST INFRASTRUCTURE ONLY).
//
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load this code, as the
// checker.  It follows the reference methods statement by statement on the plain arrays of
// include/orbx_match.h (the same POD view the GPU path takes), so the GPU kernels' parallel
// reformulations (per-node waves, wave-wide top-2, speculative greedy claims) are checked
// against the reference's sequential loops, tie rules and float expressions.
//
// Parity: the reference has no tests or fixtures for the matchers and cannot
// be built here (needs OpenCV, DBoW2 objects, MapPoint/KeyFrame).  Every rule below cites
// the line it restates; what is pinned is the restatement, not a run of the reference.
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../include/orbx_match.h"

namespace {

constexpr int TH_HIGH = 100, TH_LOW = 50, HISTO_LENGTH = 30;   // ORBmatcher.cc:37-39

// ORBmatcher::DescriptorDistance (ORBmatcher.cc:1715-1731), SWAR popcount of 8 int32 words.
int dd(const uint8_t* a8, const uint8_t* b8) {
    int32_t pa[8], pb[8];
    std::memcpy(pa, a8, 32);
    std::memcpy(pb, b8, 32);
    int dist = 0;
    for (int i = 0; i < 8; i++) {
        unsigned int v = pa[i] ^ pb[i];
        v = v - ((v >> 1) & 0x55555555);
        v = (v & 0x33333333) + ((v >> 2) & 0x33333333);
        dist += (((v + (v >> 4)) & 0xF0F0F0F) * 0x1010101) >> 24;
    }
    return dist;
}

const uint8_t* drow(const orbx_featureset* F, int i) { return F->desc + 32 * (size_t)i; }
float uright(const orbx_featureset* F, int i) { return F->u_right ? F->u_right[i] : -1.0f; }

// The rotation bin of every matcher (e.g. ORBmatcher.cc:269-275): float difference, +360
// when negative (compared as double against 0.0), round(rot * (1.0f/30)) half away from 0.
int rot_bin(float a1, float a2) {
    const float factor = 1.0f / HISTO_LENGTH;
    float rot = a1 - a2;
    if (rot < 0.0) rot += 360.0f;
    int bin = (int)std::round(rot * factor);
    if (bin == HISTO_LENGTH) bin = 0;
    return bin;
}

// ORBmatcher::ComputeThreeMaxima (ORBmatcher.cc:1669-1710).
void three_maxima(const std::vector<int>* histo, int L, int& ind1, int& ind2, int& ind3) {
    int max1 = 0, max2 = 0, max3 = 0;
    for (int i = 0; i < L; i++) {
        const int s = (int)histo[i].size();
        if (s > max1) {
            max3 = max2; max2 = max1; max1 = s;
            ind3 = ind2; ind2 = ind1; ind1 = i;
        } else if (s > max2) {
            max3 = max2; max2 = s;
            ind3 = ind2; ind2 = i;
        } else if (s > max3) {
            max3 = s; ind3 = i;
        }
    }
    if (max2 < 0.1f * (float)max1) {
        ind2 = -1; ind3 = -1;
    } else if (max3 < 0.1f * (float)max1) {
        ind3 = -1;
    }
}

// The FeatureVector as the std::map<NodeId, vector<unsigned>> it stands for.
struct FeatVecIt {
    const orbx_featureset* F;
    int j;
    bool end() const { return j >= F->n_nodes; }
    uint32_t first() const { return F->node_id[j]; }
    int size() const { return F->node_off[j + 1] - F->node_off[j]; }
    int operator[](int k) const { return F->node_feat[F->node_off[j] + k]; }
    void lower_bound(uint32_t id) {   // std::map::lower_bound over the whole map
        j = (int)(std::lower_bound(F->node_id, F->node_id + F->n_nodes, id) - F->node_id);
    }
};

// Frame::GetFeaturesInArea (Frame.cc:351-405).
std::vector<int> area_frame(const orbx_featureset* F, float x, float y, float r, int minLevel,
                            int maxLevel) {
    std::vector<int> vIndices;
    const int nMinCellX = std::max(0, (int)std::floor((x - F->min_x - r) * F->grid_inv_w));
    if (nMinCellX >= F->grid_cols) return vIndices;
    const int nMaxCellX =
        std::min(F->grid_cols - 1, (int)std::ceil((x - F->min_x + r) * F->grid_inv_w));
    if (nMaxCellX < 0) return vIndices;
    const int nMinCellY = std::max(0, (int)std::floor((y - F->min_y - r) * F->grid_inv_h));
    if (nMinCellY >= F->grid_rows) return vIndices;
    const int nMaxCellY =
        std::min(F->grid_rows - 1, (int)std::ceil((y - F->min_y + r) * F->grid_inv_h));
    if (nMaxCellY < 0) return vIndices;
    const bool bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
    for (int ix = nMinCellX; ix <= nMaxCellX; ix++)
        for (int iy = nMinCellY; iy <= nMaxCellY; iy++) {
            const int c = ix * F->grid_rows + iy;
            for (int p = F->grid_off[c]; p < F->grid_off[c + 1]; p++) {
                const int i = F->grid_feat[p];
                const orbx_keypoint& kpUn = F->keys[i];
                if (bCheckLevels) {
                    if (kpUn.octave < minLevel) continue;
                    if (maxLevel >= 0)
                        if (kpUn.octave > maxLevel) continue;
                }
                const float distx = kpUn.x - x;
                const float disty = kpUn.y - y;
                if (std::fabs(distx) < r && std::fabs(disty) < r) vIndices.push_back(i);
            }
        }
    return vIndices;
}

// KeyFrame::GetFeaturesInArea (KeyFrame.cc:583-620): same window, no level arguments.
std::vector<int> area_kf(const orbx_featureset* F, float x, float y, float r) {
    return area_frame(F, x, y, r, -1, -1);   // bCheckLevels false for (-1, -1)
}

// Removes the matches outside the three dominant rotation bins; `clear(v)` is called for
// every entry v pushed into a non-dominant bin (the reference's rotHist loops).
template <class Clear>
int rotation_filter(std::vector<int>* rotHist, Clear clear) {
    int ind1 = -1, ind2 = -1, ind3 = -1, removed = 0;
    three_maxima(rotHist, HISTO_LENGTH, ind1, ind2, ind3);
    for (int i = 0; i < HISTO_LENGTH; i++) {
        if (i == ind1 || i == ind2 || i == ind3) continue;
        for (size_t j = 0; j < rotHist[i].size(); j++) removed += clear(rotHist[i][j]);
    }
    return removed;
}

}  // namespace

extern "C" {

int oracle_descriptor_distance_m(const uint8_t* a, const uint8_t* b) { return dd(a, b); }

void oracle_three_maxima(const int32_t* counts, int L, int32_t* out3) {
    std::vector<std::vector<int>> h(L);
    for (int i = 0; i < L; i++) h[i].resize(counts[i]);
    int a = -1, b = -1, c = -1;
    three_maxima(h.data(), L, a, b, c);
    out3[0] = a; out3[1] = b; out3[2] = c;
}

// Frame::AssignFeaturesToGrid + PosInGrid (Frame.cc:243-258, 407-417): grid_off[cols*rows+1]
// and grid_feat[n] (only the features inside the grid; returns how many).
int oracle_assign_grid(const orbx_keypoint* keys, int n, int cols, int rows, float min_x,
                       float min_y, float inv_w, float inv_h, int32_t* grid_off,
                       int32_t* grid_feat) {
    std::vector<std::vector<int>> cells((size_t)cols * rows);
    for (int i = 0; i < n; i++) {
        const int posX = (int)std::round((keys[i].x - min_x) * inv_w);
        const int posY = (int)std::round((keys[i].y - min_y) * inv_h);
        if (posX < 0 || posX >= cols || posY < 0 || posY >= rows) continue;
        cells[(size_t)posX * rows + posY].push_back(i);
    }
    int k = 0;
    for (size_t c = 0; c < cells.size(); c++) {
        grid_off[c] = k;
        for (int i : cells[c]) grid_feat[k++] = i;
    }
    grid_off[cells.size()] = k;
    return k;
}

// SearchByBoW(KeyFrame*, Frame&) — ORBmatcher.cc:182-319.
int oracle_search_by_bow_kf_frame(const orbx_featureset* KF, const uint8_t* valid,
                                  const orbx_featureset* F, float nnratio, int checkOri,
                                  int32_t* match) {
    for (int i = 0; i < F->n; i++) match[i] = -1;   // :188
    std::vector<int> rotHist[HISTO_LENGTH];
    int nmatches = 0;
    FeatVecIt KFit{KF, 0}, Fit{F, 0};
    while (!KFit.end() && !Fit.end()) {   // :205
        if (KFit.first() == Fit.first()) {
            for (int iKF = 0; iKF < KFit.size(); iKF++) {
                const int realIdxKF = KFit[iKF];
                if (!valid[realIdxKF]) continue;   // :224-228
                const uint8_t* dKF = drow(KF, realIdxKF);
                int bestDist1 = 256, bestIdxF = -1, bestDist2 = 256;
                for (int iF = 0; iF < Fit.size(); iF++) {
                    const int realIdxF = Fit[iF];
                    if (match[realIdxF] >= 0) continue;   // :240
                    const int dist = dd(dKF, drow(F, realIdxF));
                    if (dist < bestDist1) {
                        bestDist2 = bestDist1; bestDist1 = dist; bestIdxF = realIdxF;
                    } else if (dist < bestDist2) {
                        bestDist2 = dist;
                    }
                }
                if (bestDist1 <= TH_LOW) {   // :259-261
                    if (static_cast<float>(bestDist1) < nnratio * static_cast<float>(bestDist2)) {
                        match[bestIdxF] = realIdxKF;
                        if (checkOri)
                            rotHist[rot_bin(KF->keys[realIdxKF].angle, F->keys[bestIdxF].angle)]
                                .push_back(bestIdxF);
                        nmatches++;
                    }
                }
            }
            KFit.j++;
            Fit.j++;
        } else if (KFit.first() < Fit.first()) {
            KFit.lower_bound(Fit.first());
        } else {
            Fit.lower_bound(KFit.first());
        }
    }
    if (checkOri)   // :298-316
        nmatches -= rotation_filter(rotHist, [&](int idx) { match[idx] = -1; return 1; });
    return nmatches;
}

// SearchByBoW(KeyFrame*, KeyFrame*) — ORBmatcher.cc:563-696.
int oracle_search_by_bow_kf_kf(const orbx_featureset* K1, const uint8_t* valid1,
                               const orbx_featureset* K2, const uint8_t* valid2, float nnratio,
                               int checkOri, int32_t* match12) {
    for (int i = 0; i < K1->n; i++) match12[i] = -1;
    std::vector<char> vbMatched2(K2->n, 0);
    std::vector<int> rotHist[HISTO_LENGTH];
    int nmatches = 0;
    FeatVecIt f1it{K1, 0}, f2it{K2, 0};
    while (!f1it.end() && !f2it.end()) {
        if (f1it.first() == f2it.first()) {
            for (int i1 = 0; i1 < f1it.size(); i1++) {
                const int idx1 = f1it[i1];
                if (!valid1[idx1]) continue;   // :599-603
                const uint8_t* d1 = drow(K1, idx1);
                int bestDist1 = 256, bestIdx2 = -1, bestDist2 = 256;
                for (int i2 = 0; i2 < f2it.size(); i2++) {
                    const int idx2 = f2it[i2];
                    if (vbMatched2[idx2] || !valid2[idx2]) continue;   // :617-621
                    const int dist = dd(d1, drow(K2, idx2));
                    if (dist < bestDist1) {
                        bestDist2 = bestDist1; bestDist1 = dist; bestIdx2 = idx2;
                    } else if (dist < bestDist2) {
                        bestDist2 = dist;
                    }
                }
                if (bestDist1 < TH_LOW) {   // :639 strict
                    if (static_cast<float>(bestDist1) < nnratio * static_cast<float>(bestDist2)) {
                        match12[idx1] = bestIdx2;
                        vbMatched2[bestIdx2] = 1;
                        if (checkOri)
                            rotHist[rot_bin(K1->keys[idx1].angle, K2->keys[bestIdx2].angle)]
                                .push_back(idx1);
                        nmatches++;
                    }
                }
            }
            f1it.j++;
            f2it.j++;
        } else if (f1it.first() < f2it.first()) {
            f1it.lower_bound(f2it.first());
        } else {
            f2it.lower_bound(f1it.first());
        }
    }
    if (checkOri)   // :675-693 (vbMatched2 is not reset)
        nmatches -= rotation_filter(rotHist, [&](int idx1) { match12[idx1] = -1; return 1; });
    return nmatches;
}

// CheckDistEpipolarLine (ORBmatcher.cc:147-167); F12 row-major.
static bool check_epipolar(const orbx_keypoint& kp1, const orbx_keypoint& kp2, const float* F12,
                           const float* sigma2) {
    const float a = kp1.x * F12[0] + kp1.y * F12[3] + F12[6];
    const float b = kp1.x * F12[1] + kp1.y * F12[4] + F12[7];
    const float c = kp1.x * F12[2] + kp1.y * F12[5] + F12[8];
    const float num = a * kp2.x + b * kp2.y + c;
    const float den = a * a + b * b;
    if (den == 0) return false;
    const float dsqr = num * num / den;
    return dsqr < 3.84 * sigma2[kp2.octave];   // double comparison
}

// SearchForTriangulation — ORBmatcher.cc:702-872.  pairs: 2 ints per match, idx1 order.
int oracle_search_for_triangulation(const orbx_featureset* K1, const uint8_t* has_mp1,
                                    const orbx_featureset* K2, const uint8_t* has_mp2,
                                    const float* F12, float ex, float ey, const float* sigma2,
                                    const float* scale, int onlyStereo, int checkOri,
                                    int32_t* match12) {
    std::vector<char> vbMatched2(K2->n, 0);   // :722, never set below
    for (int i = 0; i < K1->n; i++) match12[i] = -1;
    std::vector<int> rotHist[HISTO_LENGTH];
    int nmatches = 0;
    FeatVecIt f1it{K1, 0}, f2it{K2, 0};
    while (!f1it.end() && !f2it.end()) {
        if (f1it.first() == f2it.first()) {
            for (int i1 = 0; i1 < f1it.size(); i1++) {
                const int idx1 = f1it[i1];
                if (has_mp1[idx1]) continue;   // :749
                const bool bStereo1 = uright(K1, idx1) >= 0;
                if (onlyStereo)
                    if (!bStereo1) continue;
                const orbx_keypoint& kp1 = K1->keys[idx1];
                const uint8_t* d1 = drow(K1, idx1);
                int bestDist = TH_LOW, bestIdx2 = -1;
                for (int i2 = 0; i2 < f2it.size(); i2++) {
                    const int idx2 = f2it[i2];
                    if (vbMatched2[idx2] || has_mp2[idx2]) continue;
                    const bool bStereo2 = uright(K2, idx2) >= 0;
                    if (onlyStereo)
                        if (!bStereo2) continue;
                    const int dist = dd(d1, drow(K2, idx2));
                    if (dist > TH_LOW || dist > bestDist) continue;   // :786 (ties: last wins)
                    const orbx_keypoint& kp2 = K2->keys[idx2];
                    if (!bStereo1 && !bStereo2) {
                        const float distex = ex - kp2.x;
                        const float distey = ey - kp2.y;
                        if (distex * distex + distey * distey < 100 * scale[kp2.octave]) continue;
                    }
                    if (check_epipolar(kp1, kp2, F12, sigma2)) {
                        bestIdx2 = idx2;
                        bestDist = dist;
                    }
                }
                if (bestIdx2 >= 0) {
                    match12[idx1] = bestIdx2;
                    nmatches++;
                    if (checkOri)
                        rotHist[rot_bin(kp1.angle, K2->keys[bestIdx2].angle)].push_back(idx1);
                }
            }
            f1it.j++;
            f2it.j++;
        } else if (f1it.first() < f2it.first()) {
            f1it.lower_bound(f2it.first());
        } else {
            f2it.lower_bound(f1it.first());
        }
    }
    if (checkOri)
        nmatches -= rotation_filter(rotHist, [&](int idx1) { match12[idx1] = -1; return 1; });
    return nmatches;
}

// The projection searches (include/orbx_match.h orbx_proj_mode).  claimed may be NULL.
// qflags (may be NULL): ORBX_QF_NO_CLAIM = the query's MapPoint has no observations, so its
// match does not count as "already matched" for later queries (:90-92, :1471-1473).
// prefilter: return the accepted matches without the rotation-consistency filter.  The filter
// otherwise drops, per query, every match whose bin is not among the three maxima (with
// claims a feature has one match, so this is the reference's per-feature loop).
int oracle_search_by_projection_ex(int mode, const orbx_featureset* T, const uint8_t* claimed_in,
                                   const uint8_t* qdesc, const orbx_proj_query* Q,
                                   const uint8_t* qflags, int nq, const float* inv_sigma2,
                                   int orb_dist, float nnratio, int checkOri, int prefilter,
                                   int32_t* match_q) {
    // the per-query filter below equals the reference's per-feature loop (:1516-1535) only
    // while every feature has at most one match: LAST_FRAME with no-claim queries (a feature
    // matched twice) needs the caller's own filter (prefilter), as the C ABI requires
    if (mode == ORBX_PROJ_LAST_FRAME && checkOri && !prefilter && qflags)
        for (int iq = 0; iq < nq; iq++)
            if (qflags[iq] & ORBX_QF_NO_CLAIM) return -1;
    std::vector<char> claimed(T->n, 0);
    const bool greedy = mode <= ORBX_PROJ_KEYFRAME;
    if (claimed_in && greedy)
        for (int i = 0; i < T->n; i++) claimed[i] = claimed_in[i] != 0;
    auto claims = [&](int iq) { return !(qflags && (qflags[iq] & ORBX_QF_NO_CLAIM)); };
    std::vector<int> qbin(nq, -1);      // rotation bin of each accepted query
    std::vector<int> rotHist[HISTO_LENGTH];
    int nmatches = 0;
    for (int iq = 0; iq < nq; iq++) {
        match_q[iq] = -1;
        const orbx_proj_query& q = Q[iq];
        if (!(q.radius >= 0)) continue;
        const uint8_t* dMP = qdesc + 32 * (size_t)iq;
        if (mode == ORBX_PROJ_FRAME_MAPPOINTS) {   // ORBmatcher.cc:46-132
            const std::vector<int> vIndices =
                area_frame(T, q.u, q.v, q.radius, q.min_level, q.max_level);
            if (vIndices.empty()) continue;
            int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
            for (int idx : vIndices) {
                if (claimed[idx]) continue;   // :90-92
                if (uright(T, idx) > 0) {     // :94-99
                    const float er = std::fabs(q.ur - uright(T, idx));
                    if (er > q.radius) continue;
                }
                const int dist = dd(dMP, drow(T, idx));
                if (dist < bestDist) {
                    bestDist2 = bestDist; bestDist = dist;
                    bestLevel2 = bestLevel; bestLevel = T->keys[idx].octave;
                    bestIdx = idx;
                } else if (dist < bestDist2) {
                    bestLevel2 = T->keys[idx].octave; bestDist2 = dist;
                }
            }
            if (bestDist <= TH_HIGH) {   // :121-128
                if (bestLevel == bestLevel2 && bestDist > nnratio * bestDist2) continue;
                if (claims(iq)) claimed[bestIdx] = 1;
                match_q[iq] = bestIdx;
                nmatches++;
            }
        } else if (mode == ORBX_PROJ_LAST_FRAME || mode == ORBX_PROJ_KEYFRAME) {
            // :1415-1513 / :1556-1643
            const std::vector<int> vIndices2 =
                area_frame(T, q.u, q.v, q.radius, q.min_level, q.max_level);
            if (vIndices2.empty()) continue;
            int bestDist = 256, bestIdx2 = -1;
            for (int i2 : vIndices2) {
                if (claimed[i2]) continue;   // :1471-1473 / :1609-1610
                if (mode == ORBX_PROJ_LAST_FRAME && uright(T, i2) > 0) {   // :1475-1481
                    const float er = std::fabs(q.ur - uright(T, i2));
                    if (er > q.radius) continue;
                }
                const int dist = dd(dMP, drow(T, i2));
                if (dist < bestDist) { bestDist = dist; bestIdx2 = i2; }
            }
            const int th = mode == ORBX_PROJ_LAST_FRAME ? TH_HIGH : orb_dist;
            if (bestDist <= th) {
                if (mode == ORBX_PROJ_KEYFRAME || claims(iq)) claimed[bestIdx2] = 1;
                match_q[iq] = bestIdx2;
                nmatches++;
                if (checkOri) {
                    qbin[iq] = rot_bin(q.angle, T->keys[bestIdx2].angle);
                    rotHist[qbin[iq]].push_back(bestIdx2);
                }
            }
        } else {
            // KeyFrame grid searches: KF_SCW :393-429, FUSE :946-1024, FUSE_SCW :1107-1151,
            // SIM3 :1247-1280.
            const std::vector<int> vIndices = area_kf(T, q.u, q.v, q.radius);
            if (vIndices.empty()) continue;
            int bestDist = (mode == ORBX_PROJ_FUSE_SCW || mode == ORBX_PROJ_SIM3) ? INT_MAX : 256;
            int bestIdx = -1;
            for (int idx : vIndices) {
                if (mode == ORBX_PROJ_KF_SCW && claimed[idx]) continue;   // :406
                const orbx_keypoint& kp = T->keys[idx];
                const int kpLevel = kp.octave;
                if (kpLevel < q.pred_level - 1 || kpLevel > q.pred_level) continue;
                if (mode == ORBX_PROJ_FUSE) {   // :968-992
                    if (uright(T, idx) >= 0) {
                        const float ex = q.u - kp.x, ey = q.v - kp.y, er = q.ur - uright(T, idx);
                        const float e2 = ex * ex + ey * ey + er * er;
                        if (e2 * inv_sigma2[kpLevel] > 7.8) continue;
                    } else {
                        const float ex = q.u - kp.x, ey = q.v - kp.y;
                        const float e2 = ex * ex + ey * ey;
                        if (e2 * inv_sigma2[kpLevel] > 5.99) continue;
                    }
                }
                const int dist = dd(dMP, drow(T, idx));
                if (dist < bestDist) { bestDist = dist; bestIdx = idx; }
            }
            const int th = mode == ORBX_PROJ_SIM3 ? TH_HIGH : TH_LOW;
            if (bestDist <= th) {
                if (mode == ORBX_PROJ_KF_SCW) claimed[bestIdx] = 1;   // :427
                match_q[iq] = bestIdx;
                nmatches++;
            }
        }
    }
    if (checkOri && !prefilter && (mode == ORBX_PROJ_LAST_FRAME || mode == ORBX_PROJ_KEYFRAME)) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        three_maxima(rotHist, HISTO_LENGTH, ind1, ind2, ind3);
        for (int iq = 0; iq < nq; iq++)   // CurrentFrame.mvpMapPoints[idx] = NULL
            if (match_q[iq] >= 0 && qbin[iq] != ind1 && qbin[iq] != ind2 && qbin[iq] != ind3) {
                match_q[iq] = -1;
                nmatches--;
            }
    }
    return nmatches;
}

int oracle_search_by_projection(int mode, const orbx_featureset* T, const uint8_t* claimed_in,
                                const uint8_t* qdesc, const orbx_proj_query* Q, int nq,
                                const float* inv_sigma2, int orb_dist, float nnratio,
                                int checkOri, int32_t* match_q) {
    return oracle_search_by_projection_ex(mode, T, claimed_in, qdesc, Q, nullptr, nq, inv_sigma2,
                                          orb_dist, nnratio, checkOri, 0, match_q);
}

// SearchBySim3 — ORBmatcher.cc:1158-1382 (the two projection loops + agreement check).
int oracle_search_by_sim3(const orbx_featureset* K1, const orbx_featureset* K2,
                          const uint8_t* qdesc1, const orbx_proj_query* q12, int n1,
                          const uint8_t* qdesc2, const orbx_proj_query* q21, int n2,
                          int32_t* match12) {
    std::vector<int32_t> vnMatch1(n1), vnMatch2(n2);
    oracle_search_by_projection(ORBX_PROJ_SIM3, K2, nullptr, qdesc1, q12, n1, nullptr, 0, 0.f,
                                0, vnMatch1.data());
    oracle_search_by_projection(ORBX_PROJ_SIM3, K1, nullptr, qdesc2, q21, n2, nullptr, 0, 0.f,
                                0, vnMatch2.data());
    int nFound = 0;
    for (int i1 = 0; i1 < n1; i1++) {   // :1366-1379
        match12[i1] = -1;
        const int idx2 = vnMatch1[i1];
        if (idx2 >= 0) {
            const int idx1 = idx2 < n2 ? vnMatch2[idx2] : -1;
            if (idx1 == i1) {
                match12[i1] = idx2;
                nFound++;
            }
        }
    }
    return nFound;
}

// SearchForInitialization — ORBmatcher.cc:446-561.
int oracle_search_for_initialization(const orbx_featureset* F1, const orbx_featureset* F2,
                                     float* prev_matched, int windowSize, float nnratio,
                                     int checkOri, int32_t* vnMatches12) {
    int nmatches = 0;
    for (int i = 0; i < F1->n; i++) vnMatches12[i] = -1;
    std::vector<int> rotHist[HISTO_LENGTH];
    std::vector<int> vMatchedDistance(F2->n, INT_MAX);
    std::vector<int> vnMatches21(F2->n, -1);
    for (int i1 = 0; i1 < F1->n; i1++) {
        const orbx_keypoint kp1 = F1->keys[i1];
        const int level1 = kp1.octave;
        if (level1 > 0) continue;
        const std::vector<int> vIndices2 = area_frame(
            F2, prev_matched[2 * i1], prev_matched[2 * i1 + 1], (float)windowSize, level1, level1);
        if (vIndices2.empty()) continue;
        const uint8_t* d1 = drow(F1, i1);
        int bestDist = INT_MAX, bestDist2 = INT_MAX, bestIdx2 = -1;
        for (int i2 : vIndices2) {
            const int dist = dd(d1, drow(F2, i2));
            if (vMatchedDistance[i2] <= dist) continue;
            if (dist < bestDist) {
                bestDist2 = bestDist; bestDist = dist; bestIdx2 = i2;
            } else if (dist < bestDist2) {
                bestDist2 = dist;
            }
        }
        if (bestDist <= TH_LOW) {
            if (bestDist < (float)bestDist2 * nnratio) {
                if (vnMatches21[bestIdx2] >= 0) {
                    vnMatches12[vnMatches21[bestIdx2]] = -1;
                    nmatches--;
                }
                vnMatches12[i1] = bestIdx2;
                vnMatches21[bestIdx2] = i1;
                vMatchedDistance[bestIdx2] = bestDist;
                nmatches++;
                if (checkOri) rotHist[rot_bin(F1->keys[i1].angle, F2->keys[bestIdx2].angle)].push_back(i1);
            }
        }
    }
    if (checkOri)
        nmatches -= rotation_filter(rotHist, [&](int idx1) {
            if (vnMatches12[idx1] >= 0) {
                vnMatches12[idx1] = -1;
                return 1;
            }
            return 0;
        });
    for (int i1 = 0; i1 < F1->n; i1++)   // :555-558
        if (vnMatches12[i1] >= 0) {
            prev_matched[2 * i1] = F2->keys[vnMatches12[i1]].x;
            prev_matched[2 * i1 + 1] = F2->keys[vnMatches12[i1]].y;
        }
    return nmatches;
}

}  // extern "C"

extern "C" {
// MapPoint::ComputeDistinctiveDescriptors (src/MapPoint.cc:252-313): the row with the least
// median distance (vDists[0.5*(N-1)] of the sorted row), first on ties; -1 when N == 0.
void oracle_distinctive_descriptors(const uint8_t* desc, const int32_t* off, int np,
                                    int32_t* best) {
    for (int p = 0; p < np; ++p) {
        const int o0 = off[p];
        const size_t N = (size_t)(off[p + 1] - o0);
        if (N == 0) { best[p] = -1; continue; }
        std::vector<std::vector<float>> Distances(N, std::vector<float>(N));
        for (size_t i = 0; i < N; i++) {
            Distances[i][i] = 0;
            for (size_t j = i + 1; j < N; j++) {
                const int distij = dd(desc + 32 * (size_t)(o0 + i), desc + 32 * (size_t)(o0 + j));
                Distances[i][j] = distij;
                Distances[j][i] = distij;
            }
        }
        int BestMedian = INT_MAX, BestIdx = 0;
        for (size_t i = 0; i < N; i++) {
            std::vector<int> vDists(Distances[i].begin(), Distances[i].end());
            std::sort(vDists.begin(), vDists.end());
            const int median = vDists[0.5 * (N - 1)];
            if (median < BestMedian) {
                BestMedian = median;
                BestIdx = (int)i;
            }
        }
        best[p] = BestIdx;
    }
}

// Brute-force Hamming top-2 (SURVEY §8(b) orbx_hamming_bf_top2): the best / second loop of
// SearchByBoW (src/ORBmatcher.cc:232-256) with every database row as a candidate, in order.
// Rows [r0, r1) only, so a caller can time or check a slice of a large database.
void oracle_bf_top2(const uint8_t* q, int nq, const uint8_t* db, long long r0, long long r1,
                    int32_t* best_idx, int32_t* best_dist, int32_t* second_dist) {
    for (int i = 0; i < nq; ++i) {
        int bestDist1 = 256, bestDist2 = 256;
        long long bestIdx = -1;
        for (long long r = r0; r < r1; ++r) {
            const int dist = dd(q + 32 * (size_t)i, db + 32 * (size_t)r);
            if (dist < bestDist1) {
                bestDist2 = bestDist1;
                bestDist1 = dist;
                bestIdx = r;
            } else if (dist < bestDist2) {
                bestDist2 = dist;
            }
        }
        best_idx[i] = (int32_t)bestIdx;
        best_dist[i] = bestDist1;
        second_dist[i] = bestDist2;
    }
}
}  // extern "C"
