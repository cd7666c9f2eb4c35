// ORBmatcher.h — drop-in replacement for ORB-SLAM2's include/ORBmatcher.h (:37-128) and
// src/ORBmatcher.cc, header-only, over liborbx's C ABI (include/orbx_match.h).
//
// A maintainer copies this file over include/ORBmatcher.h, deletes src/ORBmatcher.cc from the
// ORB_SLAM2 library sources, adds <repo>/include and <repo>/integration to the include path and
// links <repo>/my_orb_slam2_amd/liborbx.so.  Frame, KeyFrame, MapPoint and every caller
// (Tracking.cc, LocalMapping.cc, LoopClosing.cc) compile unchanged: the class keeps the
// reference's constructor, public methods, static constants and return values.
//
// What runs where.  Each method keeps the reference's host-side preparation in the caller's
// own types: the cv::Mat pose arithmetic that projects a MapPoint (written with the same cv::Mat
// expressions as the reference, so OpenCV evaluates it identically), the skip tests on MapPoints,
// and the bookkeeping that writes results back into Frame / KeyFrame / MapPoint objects
// (claims, Replace / AddObservation / AddMapPoint, the rotation histogram of the projection
// searches).  The searches themselves — GetFeaturesInArea windows or FeatureVector buckets,
// DescriptorDistance over every candidate, best / second-best selection and the order-dependent
// greedy claims — run in liborbx's HIP kernels.  The Frame / KeyFrame arrays are handed over as
// orbx_featureset views built per call (mFeatVec and mGrid become CSR), so neither class needs a
// new member.
//
// GPU handles: the reference constructs an ORBmatcher on the stack at every call site (e.g.
// Tracking.cc:917 once per frame).  Creating a liborbx matcher per construction would cost a
// stream and device buffers each time, so constructed objects borrow a handle with the same
// (nnratio, checkOri) from a process-wide pool and return it in the destructor; each object
// holds its handle exclusively, so the Tracking, LocalMapping and LoopClosing threads never share
// one at the same time.
#ifndef ORBX_INTEGRATION_ORBMATCHER_H
#define ORBX_INTEGRATION_ORBMATCHER_H

#include <climits>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <mutex>
#include <set>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include <opencv2/core/core.hpp>

#include "MapPoint.h"
#include "KeyFrame.h"
#include "Frame.h"
#include "orbx_match.h"
#include "orbx_slam2_glue.h"

namespace ORB_SLAM2 {

class ORBmatcher {
public:
    // ORBmatcher.cc:41-43
    ORBmatcher(float nnratio = 0.6, bool checkOri = true)
        : mfNNratio(nnratio), mbCheckOrientation(checkOri), mpOrbx(pool_take(nnratio, checkOri)) {}
    ~ORBmatcher() { pool_give(mfNNratio, mbCheckOrientation, mpOrbx); }
    ORBmatcher(const ORBmatcher&) = delete;
    ORBmatcher& operator=(const ORBmatcher&) = delete;

    // ORBmatcher.cc:1715-1731
    static int DescriptorDistance(const cv::Mat& a, const cv::Mat& b) {
        return orbx_descriptor_distance(a.ptr(), b.ptr());
    }

    // ORBmatcher.cc:46-132 (Tracking::SearchLocalPoints).  The MapPoints' mTrack* members were
    // set by Frame::isInFrustum (or orbx_is_in_frustum).
    int SearchByProjection(Frame& F, const std::vector<MapPoint*>& vpMapPoints, const float th = 3) {
        const bool bFactor = th != 1.0;
        const size_t nq = vpMapPoints.size();
        std::vector<orbx_proj_query> q(nq);
        std::vector<uint8_t> qdesc(32 * nq), qflags(nq);
        for (size_t i = 0; i < nq; ++i) {
            MapPoint* pMP = vpMapPoints[i];
            q[i] = inactive();
            if (!pMP->mbTrackInView || pMP->isBad()) continue;   // :55-59
            const int lvl = pMP->mnTrackScaleLevel;
            float r = RadiusByViewingCos(pMP->mTrackViewCos);
            if (bFactor) r *= th;
            q[i] = {pMP->mTrackProjX, pMP->mTrackProjY, pMP->mTrackProjXR,
                    r * F.mvScaleFactors[lvl], lvl - 1, lvl, lvl, 0.f};
            std::memcpy(&qdesc[32 * i], pMP->GetDescriptor().ptr(), 32);
            qflags[i] = pMP->Observations() > 0 ? 0 : ORBX_QF_NO_CLAIM;
        }
        std::vector<uint8_t> claimed((size_t)F.N);
        for (int i = 0; i < F.N; ++i)   // :90-92
            claimed[(size_t)i] = F.mvpMapPoints[(size_t)i] && F.mvpMapPoints[(size_t)i]->Observations() > 0;
        orbx_glue::OrbxView v;
        orbx_glue::BuildView(F, v, FRAME_GRID_COLS, FRAME_GRID_ROWS);
        std::vector<int32_t> match(nq);
        run_projection(ORBX_PROJ_FRAME_MAPPOINTS, v.fs, claimed.data(), qdesc, q, qflags.data(),
                       nullptr, 0, 0, 0, match);
        int nmatches = 0;
        for (size_t i = 0; i < nq; ++i)   // :126-127
            if (match[i] >= 0) {
                F.mvpMapPoints[(size_t)match[i]] = vpMapPoints[i];
                nmatches++;
            }
        return nmatches;
    }

    // ORBmatcher.cc:1392-1538 (Tracking::TrackWithMotionModel)
    int SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, const float th,
                           const bool bMono) {
        const cv::Mat Rcw = CurrentFrame.mTcw.rowRange(0, 3).colRange(0, 3);
        const cv::Mat tcw = CurrentFrame.mTcw.rowRange(0, 3).col(3);
        const cv::Mat twc = -Rcw.t() * tcw;
        const cv::Mat Rlw = LastFrame.mTcw.rowRange(0, 3).colRange(0, 3);
        const cv::Mat tlw = LastFrame.mTcw.rowRange(0, 3).col(3);
        const cv::Mat tlc = Rlw * twc + tlw;
        const bool bForward = tlc.at<float>(2) > CurrentFrame.mb && !bMono;
        const bool bBackward = -tlc.at<float>(2) > CurrentFrame.mb && !bMono;

        const size_t nq = (size_t)LastFrame.N;
        std::vector<orbx_proj_query> q(nq);
        std::vector<uint8_t> qdesc(32 * nq), qflags(nq);
        for (size_t i = 0; i < nq; ++i) {
            q[i] = inactive();
            MapPoint* pMP = LastFrame.mvpMapPoints[i];
            if (!pMP || LastFrame.mvbOutlier[i]) continue;   // :1419-1421
            cv::Mat x3Dw = pMP->GetWorldPos();
            cv::Mat x3Dc = Rcw * x3Dw + tcw;
            const float xc = x3Dc.at<float>(0);
            const float yc = x3Dc.at<float>(1);
            const float invzc = 1.0 / x3Dc.at<float>(2);
            if (invzc < 0) continue;
            const float u = CurrentFrame.fx * xc * invzc + CurrentFrame.cx;
            const float v = CurrentFrame.fy * yc * invzc + CurrentFrame.cy;
            if (u < CurrentFrame.mnMinX || u > CurrentFrame.mnMaxX) continue;
            if (v < CurrentFrame.mnMinY || v > CurrentFrame.mnMaxY) continue;
            const int nLastOctave = LastFrame.mvKeys[i].octave;
            const float radius = th * CurrentFrame.mvScaleFactors[nLastOctave];
            int minL = nLastOctave - 1, maxL = nLastOctave + 1;   // :1453-1458
            if (bForward) {
                minL = nLastOctave;
                maxL = -1;
            } else if (bBackward) {
                minL = 0;
                maxL = nLastOctave;
            }
            q[i] = {u, v, u - CurrentFrame.mbf * invzc, radius, minL, maxL, nLastOctave,
                    LastFrame.mvKeysUn[i].angle};
            std::memcpy(&qdesc[32 * i], pMP->GetDescriptor().ptr(), 32);
            qflags[i] = pMP->Observations() > 0 ? 0 : ORBX_QF_NO_CLAIM;
        }
        std::vector<uint8_t> claimed((size_t)CurrentFrame.N);
        for (int i = 0; i < CurrentFrame.N; ++i)   // :1471-1473
            claimed[(size_t)i] = CurrentFrame.mvpMapPoints[(size_t)i] &&
                                 CurrentFrame.mvpMapPoints[(size_t)i]->Observations() > 0;
        orbx_glue::OrbxView v;
        orbx_glue::BuildView(CurrentFrame, v, FRAME_GRID_COLS, FRAME_GRID_ROWS);
        std::vector<int32_t> match(nq);
        run_projection(ORBX_PROJ_LAST_FRAME, v.fs, claimed.data(), qdesc, q, qflags.data(),
                       nullptr, 0, 0, ORBX_PROJ_PREFILTER, match);
        // :1494-1535: the matches in MapPoint order, then the rotation-consistency filter over
        // the frame features (a feature matched twice sits in the histogram twice)
        std::vector<int> rotHist[HISTO_LENGTH];
        int nmatches = 0;
        for (size_t i = 0; i < nq; ++i) {
            const int b = match[i];
            if (b < 0) continue;
            CurrentFrame.mvpMapPoints[(size_t)b] = LastFrame.mvpMapPoints[i];
            nmatches++;
            if (mbCheckOrientation)
                rotHist[RotationBin(LastFrame.mvKeysUn[i].angle, CurrentFrame.mvKeysUn[(size_t)b].angle)].push_back(b);
        }
        if (mbCheckOrientation)
            nmatches -= DropOutsideThreeMaxima(rotHist, [&](int idx) {
                CurrentFrame.mvpMapPoints[(size_t)idx] = static_cast<MapPoint*>(NULL);
            });
        return nmatches;
    }

    // ORBmatcher.cc:1540-1667 (Tracking::Relocalization)
    int SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF, const std::set<MapPoint*>& sAlreadyFound,
                           const float th, const int ORBdist) {
        const cv::Mat Rcw = CurrentFrame.mTcw.rowRange(0, 3).colRange(0, 3);
        const cv::Mat tcw = CurrentFrame.mTcw.rowRange(0, 3).col(3);
        const cv::Mat Ow = -Rcw.t() * tcw;
        const std::vector<MapPoint*> vpMPs = pKF->GetMapPointMatches();
        const size_t nq = vpMPs.size();
        std::vector<orbx_proj_query> q(nq);
        std::vector<uint8_t> qdesc(32 * nq);
        for (size_t i = 0; i < nq; ++i) {
            q[i] = inactive();
            MapPoint* pMP = vpMPs[i];
            if (!pMP || pMP->isBad() || sAlreadyFound.count(pMP)) continue;   // :1560-1562
            cv::Mat x3Dw = pMP->GetWorldPos();
            cv::Mat x3Dc = Rcw * x3Dw + tcw;
            const float xc = x3Dc.at<float>(0);
            const float yc = x3Dc.at<float>(1);
            const float invzc = 1.0 / x3Dc.at<float>(2);
            const float u = CurrentFrame.fx * xc * invzc + CurrentFrame.cx;
            const float v = CurrentFrame.fy * yc * invzc + CurrentFrame.cy;
            if (u < CurrentFrame.mnMinX || u > CurrentFrame.mnMaxX) continue;
            if (v < CurrentFrame.mnMinY || v > CurrentFrame.mnMaxY) continue;
            cv::Mat PO = x3Dw - Ow;
            float dist3D = cv::norm(PO);
            const float maxDistance = pMP->GetMaxDistanceInvariance();
            const float minDistance = pMP->GetMinDistanceInvariance();
            if (dist3D < minDistance || dist3D > maxDistance) continue;
            const int nPredictedLevel = pMP->PredictScale(dist3D, &CurrentFrame);
            const float radius = th * CurrentFrame.mvScaleFactors[nPredictedLevel];
            q[i] = {u, v, 0.f, radius, nPredictedLevel - 1, nPredictedLevel + 1, nPredictedLevel,
                    pKF->mvKeysUn[i].angle};
            std::memcpy(&qdesc[32 * i], pMP->GetDescriptor().ptr(), 32);
        }
        std::vector<uint8_t> claimed((size_t)CurrentFrame.N);
        for (int i = 0; i < CurrentFrame.N; ++i)   // :1609-1610
            claimed[(size_t)i] = CurrentFrame.mvpMapPoints[(size_t)i] != nullptr;
        orbx_glue::OrbxView v;
        orbx_glue::BuildView(CurrentFrame, v, FRAME_GRID_COLS, FRAME_GRID_ROWS);
        std::vector<int32_t> match(nq);
        run_projection(ORBX_PROJ_KEYFRAME, v.fs, claimed.data(), qdesc, q, nullptr, nullptr, 0,
                       ORBdist, ORBX_PROJ_PREFILTER, match);
        std::vector<int> rotHist[HISTO_LENGTH];
        int nmatches = 0;
        for (size_t i = 0; i < nq; ++i) {   // :1623-1639
            const int b = match[i];
            if (b < 0) continue;
            CurrentFrame.mvpMapPoints[(size_t)b] = vpMPs[i];
            nmatches++;
            if (mbCheckOrientation)
                rotHist[RotationBin(pKF->mvKeysUn[i].angle, CurrentFrame.mvKeysUn[(size_t)b].angle)].push_back(b);
        }
        if (mbCheckOrientation)
            nmatches -= DropOutsideThreeMaxima(rotHist, [&](int idx) {
                CurrentFrame.mvpMapPoints[(size_t)idx] = NULL;
            });
        return nmatches;
    }

    // ORBmatcher.cc:321-434 (LoopClosing::ComputeSim3)
    int SearchByProjection(KeyFrame* pKF, cv::Mat Scw, const std::vector<MapPoint*>& vpPoints,
                           std::vector<MapPoint*>& vpMatched, int th) {
        const float& fx = pKF->fx;
        const float& fy = pKF->fy;
        const float& cx = pKF->cx;
        const float& cy = pKF->cy;
        cv::Mat sRcw = Scw.rowRange(0, 3).colRange(0, 3);
        const float scw = std::sqrt(sRcw.row(0).dot(sRcw.row(0)));
        cv::Mat Rcw = sRcw / scw;
        cv::Mat tcw = Scw.rowRange(0, 3).col(3) / scw;
        cv::Mat Ow = -Rcw.t() * tcw;
        std::set<MapPoint*> spAlreadyFound(vpMatched.begin(), vpMatched.end());
        spAlreadyFound.erase(static_cast<MapPoint*>(NULL));

        const size_t nq = vpPoints.size();
        std::vector<orbx_proj_query> q(nq);
        std::vector<uint8_t> qdesc(32 * nq);
        for (size_t iMP = 0; iMP < nq; ++iMP) {
            q[iMP] = inactive();
            MapPoint* pMP = vpPoints[iMP];
            if (pMP->isBad() || spAlreadyFound.count(pMP)) continue;   // :348-349
            cv::Mat p3Dw = pMP->GetWorldPos();
            cv::Mat p3Dc = Rcw * p3Dw + tcw;
            if (p3Dc.at<float>(2) < 0.0) continue;
            const float invz = 1 / p3Dc.at<float>(2);
            const float x = p3Dc.at<float>(0) * invz;
            const float y = p3Dc.at<float>(1) * invz;
            const float u = fx * x + cx;
            const float v = fy * y + cy;
            if (!pKF->IsInImage(u, v)) continue;
            const float maxDistance = pMP->GetMaxDistanceInvariance();
            const float minDistance = pMP->GetMinDistanceInvariance();
            cv::Mat PO = p3Dw - Ow;
            const float dist = cv::norm(PO);
            if (dist < minDistance || dist > maxDistance) continue;
            cv::Mat Pn = pMP->GetNormal();
            if (PO.dot(Pn) < 0.5 * dist) continue;
            const int nPredictedLevel = pMP->PredictScale(dist, pKF);
            const float radius = th * pKF->mvScaleFactors[nPredictedLevel];
            q[iMP] = {u, v, 0.f, radius, -1, -1, nPredictedLevel, 0.f};
            std::memcpy(&qdesc[32 * iMP], pMP->GetDescriptor().ptr(), 32);
        }
        std::vector<uint8_t> claimed((size_t)pKF->N);
        for (int i = 0; i < pKF->N; ++i) claimed[(size_t)i] = vpMatched[(size_t)i] != nullptr;   // :406
        orbx_glue::OrbxView v;
        orbx_glue::BuildView(*pKF, v, pKF->mnGridCols, pKF->mnGridRows);
        std::vector<int32_t> match(nq);
        run_projection(ORBX_PROJ_KF_SCW, v.fs, claimed.data(), qdesc, q, nullptr, nullptr, 0, 0, 0,
                       match);
        int nmatches = 0;
        for (size_t iMP = 0; iMP < nq; ++iMP)   // :425-429
            if (match[iMP] >= 0) {
                vpMatched[(size_t)match[iMP]] = vpPoints[iMP];
                nmatches++;
            }
        return nmatches;
    }

    // ORBmatcher.cc:182-319 (Tracking::TrackReferenceKeyFrame, Relocalization)
    int SearchByBoW(KeyFrame* pKF, Frame& F, std::vector<MapPoint*>& vpMapPointMatches) {
        orbx_glue::OrbxView kv, fv;
        orbx_glue::BuildView(*pKF, kv, 0, 0);
        orbx_glue::BuildView(F, fv, 0, 0);
        return orbx_glue::SearchByBoW(mpOrbx, pKF, kv, F, fv, vpMapPointMatches);
    }

    // ORBmatcher.cc:563-696 (LoopClosing::ComputeSim3)
    int SearchByBoW(KeyFrame* pKF1, KeyFrame* pKF2, std::vector<MapPoint*>& vpMatches12) {
        const std::vector<MapPoint*> vpMapPoints1 = pKF1->GetMapPointMatches();
        const std::vector<MapPoint*> vpMapPoints2 = pKF2->GetMapPointMatches();
        std::vector<uint8_t> valid1(vpMapPoints1.size()), valid2(vpMapPoints2.size());
        for (size_t i = 0; i < valid1.size(); ++i) valid1[i] = vpMapPoints1[i] && !vpMapPoints1[i]->isBad();
        for (size_t i = 0; i < valid2.size(); ++i) valid2[i] = vpMapPoints2[i] && !vpMapPoints2[i]->isBad();
        orbx_glue::OrbxView v1, v2;
        orbx_glue::BuildView(*pKF1, v1, 0, 0);
        orbx_glue::BuildView(*pKF2, v2, 0, 0);
        std::vector<int32_t> match(vpMapPoints1.size() + 1);
        int32_t n = 0;
        orbx_glue::check(orbx_search_by_bow_kf_kf(mpOrbx, &v1.fs, valid1.data(), &v2.fs, valid2.data(),
                                                  match.data(), &n),
                         "orbx_search_by_bow_kf_kf");
        vpMatches12 = std::vector<MapPoint*>(vpMapPoints1.size(), static_cast<MapPoint*>(NULL));
        for (size_t i = 0; i < vpMapPoints1.size(); ++i)
            if (match[i] >= 0) vpMatches12[i] = vpMapPoints2[(size_t)match[i]];
        return n;
    }

    // ORBmatcher.cc:446-561 (Tracking::MonocularInitialization)
    int SearchForInitialization(Frame& F1, Frame& F2, std::vector<cv::Point2f>& vbPrevMatched,
                                std::vector<int>& vnMatches12, int windowSize = 10) {
        static_assert(sizeof(cv::Point2f) == 2 * sizeof(float), "cv::Point2f layout");
        vnMatches12 = std::vector<int>(F1.mvKeysUn.size(), -1);
        orbx_glue::OrbxView v1, v2;
        orbx_glue::BuildView(F1, v1, FRAME_GRID_COLS, FRAME_GRID_ROWS);
        orbx_glue::BuildView(F2, v2, FRAME_GRID_COLS, FRAME_GRID_ROWS);
        std::vector<int32_t> match(vnMatches12.size() + 1);
        int32_t n = 0;
        orbx_glue::check(orbx_search_for_initialization(mpOrbx, &v1.fs, &v2.fs,
                                                        reinterpret_cast<float*>(vbPrevMatched.data()),
                                                        windowSize, match.data(), &n),
                         "orbx_search_for_initialization");   // updates vbPrevMatched (:555-558)
        for (size_t i = 0; i < vnMatches12.size(); ++i) vnMatches12[i] = match[i];
        return n;
    }

    // ORBmatcher.cc:702-872 (LocalMapping::CreateNewMapPoints)
    int SearchForTriangulation(KeyFrame* pKF1, KeyFrame* pKF2, cv::Mat F12,
                               std::vector<std::pair<size_t, size_t>>& vMatchedPairs,
                               const bool bOnlyStereo) {
        cv::Mat Cw = pKF1->GetCameraCenter();   // the epipole, :709-715
        cv::Mat R2w = pKF2->GetRotation();
        cv::Mat t2w = pKF2->GetTranslation();
        cv::Mat C2 = R2w * Cw + t2w;
        const float invz = 1.0f / C2.at<float>(2);
        const float ex = pKF2->fx * C2.at<float>(0) * invz + pKF2->cx;
        const float ey = pKF2->fy * C2.at<float>(1) * invz + pKF2->cy;
        float f12[9];
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) f12[3 * r + c] = F12.at<float>(r, c);
        std::vector<uint8_t> mp1((size_t)pKF1->N), mp2((size_t)pKF2->N);
        for (int i = 0; i < pKF1->N; ++i) mp1[(size_t)i] = pKF1->GetMapPoint((size_t)i) != nullptr;
        for (int i = 0; i < pKF2->N; ++i) mp2[(size_t)i] = pKF2->GetMapPoint((size_t)i) != nullptr;
        orbx_glue::OrbxView v1, v2;
        orbx_glue::BuildView(*pKF1, v1, 0, 0);
        orbx_glue::BuildView(*pKF2, v2, 0, 0);
        std::vector<int32_t> pairs(2 * (size_t)pKF1->N + 2);
        int32_t n = 0;
        orbx_glue::check(orbx_search_for_triangulation(
                             mpOrbx, &v1.fs, mp1.data(), &v2.fs, mp2.data(), f12, ex, ey,
                             pKF2->mvLevelSigma2.data(), pKF2->mvScaleFactors.data(),
                             (int32_t)pKF2->mvScaleFactors.size(), bOnlyStereo, pairs.data(),
                             pKF1->N, &n),
                         "orbx_search_for_triangulation");
        vMatchedPairs.clear();
        vMatchedPairs.reserve((size_t)n);
        for (int k = 0; k < n; ++k)
            vMatchedPairs.push_back(std::make_pair((size_t)pairs[2 * (size_t)k], (size_t)pairs[2 * (size_t)k + 1]));
        return n;
    }

    // ORBmatcher.cc:1158-1382 (LoopClosing::ComputeSim3)
    int SearchBySim3(KeyFrame* pKF1, KeyFrame* pKF2, std::vector<MapPoint*>& vpMatches12,
                     const float& s12, const cv::Mat& R12, const cv::Mat& t12, const float th) {
        const float& fx = pKF1->fx;
        const float& fy = pKF1->fy;
        const float& cx = pKF1->cx;
        const float& cy = pKF1->cy;
        cv::Mat R1w = pKF1->GetRotation();
        cv::Mat t1w = pKF1->GetTranslation();
        cv::Mat R2w = pKF2->GetRotation();
        cv::Mat t2w = pKF2->GetTranslation();
        cv::Mat sR12 = s12 * R12;
        cv::Mat sR21 = (1.0 / s12) * R12.t();
        cv::Mat t21 = -sR21 * t12;
        const std::vector<MapPoint*> vpMapPoints1 = pKF1->GetMapPointMatches();
        const int N1 = (int)vpMapPoints1.size();
        const std::vector<MapPoint*> vpMapPoints2 = pKF2->GetMapPointMatches();
        const int N2 = (int)vpMapPoints2.size();
        std::vector<bool> vbAlreadyMatched1((size_t)N1, false), vbAlreadyMatched2((size_t)N2, false);
        for (int i = 0; i < N1; i++) {   // :1188-1198
            MapPoint* pMP = vpMatches12[(size_t)i];
            if (!pMP) continue;
            vbAlreadyMatched1[(size_t)i] = true;
            const int idx2 = pMP->GetIndexInKeyFrame(pKF2);
            if (idx2 >= 0 && idx2 < N2) vbAlreadyMatched2[(size_t)idx2] = true;
        }
        // one projection per direction (:1204-1281 KF1 -> KF2 with sR21, t21; :1284-1361 KF2 ->
        // KF1 with sR12, t12), both through pKF1's intrinsics as in the reference
        auto project = [&](const std::vector<MapPoint*>& pts, const std::vector<bool>& done,
                           const cv::Mat& Rw, const cv::Mat& tw, const cv::Mat& sR, const cv::Mat& t,
                           KeyFrame* pTo, std::vector<orbx_proj_query>& q, std::vector<uint8_t>& d) {
            q.assign(pts.size(), inactive());
            d.assign(32 * pts.size(), 0);
            for (size_t i = 0; i < pts.size(); ++i) {
                MapPoint* pMP = pts[i];
                if (!pMP || done[i] || pMP->isBad()) continue;
                cv::Mat p3Dw = pMP->GetWorldPos();
                cv::Mat p3Dc_from = Rw * p3Dw + tw;
                cv::Mat p3Dc_to = sR * p3Dc_from + t;
                if (p3Dc_to.at<float>(2) < 0.0) continue;
                const float invz = 1.0 / p3Dc_to.at<float>(2);
                const float x = p3Dc_to.at<float>(0) * invz;
                const float y = p3Dc_to.at<float>(1) * invz;
                const float u = fx * x + cx;
                const float v = fy * y + cy;
                if (!pTo->IsInImage(u, v)) continue;
                const float maxDistance = pMP->GetMaxDistanceInvariance();
                const float minDistance = pMP->GetMinDistanceInvariance();
                const float dist3D = cv::norm(p3Dc_to);
                if (dist3D < minDistance || dist3D > maxDistance) continue;
                const int nPredictedLevel = pMP->PredictScale(dist3D, pTo);
                const float radius = th * pTo->mvScaleFactors[nPredictedLevel];
                q[i] = {u, v, 0.f, radius, -1, -1, nPredictedLevel, 0.f};
                std::memcpy(&d[32 * i], pMP->GetDescriptor().ptr(), 32);
            }
        };
        std::vector<orbx_proj_query> q12, q21;
        std::vector<uint8_t> d1, d2;
        project(vpMapPoints1, vbAlreadyMatched1, R1w, t1w, sR21, t21, pKF2, q12, d1);
        project(vpMapPoints2, vbAlreadyMatched2, R2w, t2w, sR12, t12, pKF1, q21, d2);
        orbx_glue::OrbxView v1, v2;
        orbx_glue::BuildView(*pKF1, v1, pKF1->mnGridCols, pKF1->mnGridRows);
        orbx_glue::BuildView(*pKF2, v2, pKF2->mnGridCols, pKF2->mnGridRows);
        std::vector<int32_t> match((size_t)N1 + 1);
        int32_t nFound = 0;
        orbx_glue::check(orbx_search_by_sim3(mpOrbx, &v1.fs, &v2.fs, d1.data(), q12.data(), N1,
                                             d2.data(), q21.data(), N2, match.data(), &nFound),
                         "orbx_search_by_sim3");
        for (int i1 = 0; i1 < N1; i1++)   // :1366-1379
            if (match[(size_t)i1] >= 0) vpMatches12[(size_t)i1] = vpMapPoints2[(size_t)match[(size_t)i1]];
        return nFound;
    }

    // ORBmatcher.cc:879-1029 (LocalMapping::SearchInNeighbors)
    int Fuse(KeyFrame* pKF, const std::vector<MapPoint*>& vpMapPoints, const float th = 3.0) {
        cv::Mat Rcw = pKF->GetRotation();
        cv::Mat tcw = pKF->GetTranslation();
        const float& fx = pKF->fx;
        const float& fy = pKF->fy;
        const float& cx = pKF->cx;
        const float& cy = pKF->cy;
        const float& bf = pKF->mbf;
        cv::Mat Ow = pKF->GetCameraCenter();
        const size_t nq = vpMapPoints.size();
        std::vector<orbx_proj_query> q(nq);
        std::vector<uint8_t> qdesc(32 * nq);
        for (size_t i = 0; i < nq; ++i) {
            q[i] = inactive();
            MapPoint* pMP = vpMapPoints[i];
            // skipped now => skipped at its turn: isBad stays set and a good MapPoint only gains
            // observations; the test is repeated at its turn below
            if (!pMP || pMP->isBad() || pMP->IsInKeyFrame(pKF)) continue;
            cv::Mat p3Dw = pMP->GetWorldPos();
            cv::Mat p3Dc = Rcw * p3Dw + tcw;
            if (p3Dc.at<float>(2) < 0.0f) continue;
            const float invz = 1 / p3Dc.at<float>(2);
            const float x = p3Dc.at<float>(0) * invz;
            const float y = p3Dc.at<float>(1) * invz;
            const float u = fx * x + cx;
            const float v = fy * y + cy;
            if (!pKF->IsInImage(u, v)) continue;
            const float ur = u - bf * invz;
            const float maxDistance = pMP->GetMaxDistanceInvariance();
            const float minDistance = pMP->GetMinDistanceInvariance();
            cv::Mat PO = p3Dw - Ow;
            const float dist3D = cv::norm(PO);
            if (dist3D < minDistance || dist3D > maxDistance) continue;
            cv::Mat Pn = pMP->GetNormal();
            if (PO.dot(Pn) < 0.5 * dist3D) continue;
            const int nPredictedLevel = pMP->PredictScale(dist3D, pKF);
            const float radius = th * pKF->mvScaleFactors[nPredictedLevel];
            q[i] = {u, v, ur, radius, -1, -1, nPredictedLevel, 0.f};
            std::memcpy(&qdesc[32 * i], pMP->GetDescriptor().ptr(), 32);
        }
        orbx_glue::OrbxView v;
        orbx_glue::BuildView(*pKF, v, pKF->mnGridCols, pKF->mnGridRows);
        std::vector<int32_t> match(nq);
        run_projection(ORBX_PROJ_FUSE, v.fs, nullptr, qdesc, q, nullptr,
                       pKF->mvInvLevelSigma2.data(), (int32_t)pKF->mvInvLevelSigma2.size(), 0, 0,
                       match);
        int nFused = 0;
        for (size_t i = 0; i < nq; ++i) {   // :1005-1025, in MapPoint order
            if (match[i] < 0) continue;
            MapPoint* pMP = vpMapPoints[i];
            if (pMP->isBad() || pMP->IsInKeyFrame(pKF)) continue;
            const size_t bestIdx = (size_t)match[i];
            MapPoint* pMPinKF = pKF->GetMapPoint(bestIdx);
            if (pMPinKF) {
                if (!pMPinKF->isBad()) {
                    if (pMPinKF->Observations() > pMP->Observations())
                        pMP->Replace(pMPinKF);
                    else
                        pMPinKF->Replace(pMP);
                }
            } else {
                pMP->AddObservation(pKF, bestIdx);
                pKF->AddMapPoint(pMP, bestIdx);
            }
            nFused++;
        }
        return nFused;
    }

    // ORBmatcher.cc:1033-1156 (LoopClosing::SearchAndFuse)
    int Fuse(KeyFrame* pKF, cv::Mat Scw, const std::vector<MapPoint*>& vpPoints, float th,
             std::vector<MapPoint*>& vpReplacePoint) {
        const float& fx = pKF->fx;
        const float& fy = pKF->fy;
        const float& cx = pKF->cx;
        const float& cy = pKF->cy;
        cv::Mat sRcw = Scw.rowRange(0, 3).colRange(0, 3);
        const float scw = std::sqrt(sRcw.row(0).dot(sRcw.row(0)));
        cv::Mat Rcw = sRcw / scw;
        cv::Mat tcw = Scw.rowRange(0, 3).col(3) / scw;
        cv::Mat Ow = -Rcw.t() * tcw;
        const std::set<MapPoint*> spAlreadyFound = pKF->GetMapPoints();
        const size_t nq = vpPoints.size();
        std::vector<orbx_proj_query> q(nq);
        std::vector<uint8_t> qdesc(32 * nq);
        for (size_t iMP = 0; iMP < nq; ++iMP) {
            q[iMP] = inactive();
            MapPoint* pMP = vpPoints[iMP];
            if (pMP->isBad() || spAlreadyFound.count(pMP)) continue;   // :1061-1062
            cv::Mat p3Dw = pMP->GetWorldPos();
            cv::Mat p3Dc = Rcw * p3Dw + tcw;
            if (p3Dc.at<float>(2) < 0.0f) continue;
            const float invz = 1.0 / p3Dc.at<float>(2);
            const float x = p3Dc.at<float>(0) * invz;
            const float y = p3Dc.at<float>(1) * invz;
            const float u = fx * x + cx;
            const float v = fy * y + cy;
            if (!pKF->IsInImage(u, v)) continue;
            const float maxDistance = pMP->GetMaxDistanceInvariance();
            const float minDistance = pMP->GetMinDistanceInvariance();
            cv::Mat PO = p3Dw - Ow;
            const float dist3D = cv::norm(PO);
            if (dist3D < minDistance || dist3D > maxDistance) continue;
            cv::Mat Pn = pMP->GetNormal();
            if (PO.dot(Pn) < 0.5 * dist3D) continue;
            const int nPredictedLevel = pMP->PredictScale(dist3D, pKF);
            const float radius = th * pKF->mvScaleFactors[nPredictedLevel];
            q[iMP] = {u, v, 0.f, radius, -1, -1, nPredictedLevel, 0.f};
            std::memcpy(&qdesc[32 * iMP], pMP->GetDescriptor().ptr(), 32);
        }
        orbx_glue::OrbxView v;
        orbx_glue::BuildView(*pKF, v, pKF->mnGridCols, pKF->mnGridRows);
        std::vector<int32_t> match(nq);
        run_projection(ORBX_PROJ_FUSE_SCW, v.fs, nullptr, qdesc, q, nullptr, nullptr, 0, 0, 0, match);
        int nFused = 0;
        for (size_t iMP = 0; iMP < nq; ++iMP) {   // :1138-1152, in MapPoint order
            if (match[iMP] < 0) continue;
            MapPoint* pMP = vpPoints[iMP];
            if (pMP->isBad()) continue;
            const size_t bestIdx = (size_t)match[iMP];
            MapPoint* pMPinKF = pKF->GetMapPoint(bestIdx);
            if (pMPinKF) {
                if (!pMPinKF->isBad()) vpReplacePoint[iMP] = pMPinKF;
            } else {
                pMP->AddObservation(pKF, bestIdx);
                pKF->AddMapPoint(pMP, bestIdx);
            }
            nFused++;
        }
        return nFused;
    }

public:
    static const int TH_LOW = ORBX_TH_LOW;              // ORBmatcher.cc:37-39
    static const int TH_HIGH = ORBX_TH_HIGH;
    static const int HISTO_LENGTH = ORBX_HISTO_LENGTH;

protected:
    // ORBmatcher.cc:147-167 (kept for subclasses; SearchForTriangulation runs it on the GPU)
    bool CheckDistEpipolarLine(const cv::KeyPoint& kp1, const cv::KeyPoint& kp2, const cv::Mat& F12,
                               const KeyFrame* pKF2) {
        const float a = kp1.pt.x * F12.at<float>(0, 0) + kp1.pt.y * F12.at<float>(1, 0) + F12.at<float>(2, 0);
        const float b = kp1.pt.x * F12.at<float>(0, 1) + kp1.pt.y * F12.at<float>(1, 1) + F12.at<float>(2, 1);
        const float c = kp1.pt.x * F12.at<float>(0, 2) + kp1.pt.y * F12.at<float>(1, 2) + F12.at<float>(2, 2);
        const float num = a * kp2.pt.x + b * kp2.pt.y + c;
        const float den = a * a + b * b;
        if (den == 0) return false;
        return num * num / den < 3.84 * pKF2->mvLevelSigma2[(size_t)kp2.octave];
    }
    // ORBmatcher.cc:134-140
    float RadiusByViewingCos(const float& viewCos) { return viewCos > 0.998 ? 2.5 : 4.0; }
    // ORBmatcher.cc:1669-1710
    void ComputeThreeMaxima(std::vector<int>* histo, const int L, int& ind1, int& ind2, int& ind3) {
        std::vector<int32_t> counts((size_t)L);
        for (int i = 0; i < L; ++i) counts[(size_t)i] = (int32_t)histo[i].size();
        orbx_compute_three_maxima(counts.data(), L, &ind1, &ind2, &ind3);
    }

    float mfNNratio;
    bool mbCheckOrientation;

private:
    orbx_matcher* mpOrbx;

    static orbx_proj_query inactive() { return {0.f, 0.f, 0.f, -1.f, -1, -1, 0, 0.f}; }

    // the rotation bin of ORBmatcher.cc:269-276 (factor = 1/HISTO_LENGTH)
    static int RotationBin(float a1, float a2) {
        float rot = a1 - a2;
        if (rot < 0.0) rot += 360.0f;
        int bin = (int)std::round(rot * (1.0f / HISTO_LENGTH));
        if (bin == HISTO_LENGTH) bin = 0;
        return bin;
    }
    // the rotation-consistency loop of :1516-1535: clears every entry outside the three largest
    // bins; returns how many it cleared
    template <class Clear>
    int DropOutsideThreeMaxima(std::vector<int>* rotHist, Clear clear) {
        int ind1 = -1, ind2 = -1, ind3 = -1, dropped = 0;
        ComputeThreeMaxima(rotHist, HISTO_LENGTH, ind1, ind2, ind3);
        for (int i = 0; i < HISTO_LENGTH; i++) {
            if (i == ind1 || i == ind2 || i == ind3) continue;
            for (int idx : rotHist[i]) {
                clear(idx);
                dropped++;
            }
        }
        return dropped;
    }

    void run_projection(int mode, const orbx_featureset& target, const uint8_t* claimed,
                        const std::vector<uint8_t>& qdesc, const std::vector<orbx_proj_query>& q,
                        const uint8_t* qflags, const float* inv_sigma2, int32_t nlevels,
                        int32_t orb_dist, int32_t flags, std::vector<int32_t>& match) {
        int32_t n = 0;
        match.assign(q.size(), -1);
        if (q.empty()) return;
        orbx_glue::check(orbx_search_by_projection_ex(mpOrbx, mode, &target, claimed, qdesc.data(),
                                                      q.data(), qflags, (int32_t)q.size(),
                                                      inv_sigma2, nlevels, orb_dist, flags,
                                                      match.data(), &n),
                         "orbx_search_by_projection_ex");
    }

    // the handle pool (see the file comment)
    typedef std::pair<uint32_t, bool> PoolKey;
    static std::mutex& pool_mutex() {
        static std::mutex m;
        return m;
    }
    static std::multimap<PoolKey, orbx_matcher*>& pool() {
        static std::multimap<PoolKey, orbx_matcher*> p;
        return p;
    }
    static PoolKey pool_key(float nnratio, bool checkOri) {
        uint32_t bits;
        std::memcpy(&bits, &nnratio, 4);
        return PoolKey(bits, checkOri);
    }
    static orbx_matcher* pool_take(float nnratio, bool checkOri) {
        {
            std::lock_guard<std::mutex> lk(pool_mutex());
            auto it = pool().find(pool_key(nnratio, checkOri));
            if (it != pool().end()) {
                orbx_matcher* m = it->second;
                pool().erase(it);
                return m;
            }
        }
        orbx_matcher* m = nullptr;
        const orbx_matcher_params p = {nnratio, checkOri ? 1 : 0, 0};
        orbx_glue::check(orbx_matcher_create(&p, &m), "orbx_matcher_create");
        return m;
    }
    static void pool_give(float nnratio, bool checkOri, orbx_matcher* m) {
        if (!m) return;
        std::lock_guard<std::mutex> lk(pool_mutex());
        pool().insert(std::make_pair(pool_key(nnratio, checkOri), m));
    }
};

}  // namespace ORB_SLAM2

#endif  // ORBX_INTEGRATION_ORBMATCHER_H
