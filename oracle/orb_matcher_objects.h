// orb_matcher_objects.h — TEST INFRASTRUCTURE (the oracle): a CPU restatement of every public
// method of ORB-SLAM2's ORBmatcher (src/ORBmatcher.cc) at the level of the reference's own
// objects: it takes Frame / KeyFrame / MapPoint, walks GetFeaturesInArea windows and FeatureVector
// buckets itself, computes DescriptorDistance on every candidate and writes the results back
// exactly as the reference does.  tests/native/matcher_test.cpp runs it beside the drop-in
// integration/ORBmatcher.h (whose searches run on the GPU) on identical copies of synthetic
// scenes and compares outputs and every state change.  Nothing in the product includes this
// file.  PARITY against the reference is by restatement (the reference cannot be built here,
// DESIGN.md §2); each method cites the lines it follows.
#ifndef ORBX_ORACLE_MATCHER_OBJECTS_H
#define ORBX_ORACLE_MATCHER_OBJECTS_H

#include <climits>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <set>
#include <utility>
#include <vector>

#include <opencv2/core/core.hpp>

namespace orbx_oracle {

template <class Frame, class KeyFrame, class MapPoint>
class ObjectMatcher {
public:
    static constexpr int kLow = 50, kHigh = 100, kBins = 30;   // ORBmatcher.cc:37-39

    ObjectMatcher(float nnratio = 0.6f, bool checkOri = true) : ratio_(nnratio), ori_(checkOri) {}

    // :1715-1731, the SWAR popcount over eight 32-bit words
    static int Distance(const cv::Mat& a, const cv::Mat& b) {
        const uint8_t* pa = a.ptr();
        const uint8_t* pb = b.ptr();
        int d = 0;
        for (int w = 0; w < 8; ++w) {
            uint32_t x, y;
            std::memcpy(&x, pa + 4 * w, 4);
            std::memcpy(&y, pb + 4 * w, 4);
            uint32_t v = x ^ y;
            v = v - ((v >> 1) & 0x55555555u);
            v = (v & 0x33333333u) + ((v >> 2) & 0x33333333u);
            d += (int)((((v + (v >> 4)) & 0x0F0F0F0Fu) * 0x01010101u) >> 24);
        }
        return d;
    }

    // :46-132
    int ProjectLocalMap(Frame& F, const std::vector<MapPoint*>& points, float th) {
        int n = 0;
        for (MapPoint* pMP : points) {
            if (!pMP->mbTrackInView || pMP->isBad()) continue;
            const int lvl = pMP->mnTrackScaleLevel;
            float r = pMP->mTrackViewCos > 0.998 ? 2.5f : 4.0f;
            if (th != 1.0) r *= th;
            const float win = r * F.mvScaleFactors[lvl];
            const std::vector<size_t> cand = F.GetFeaturesInArea(pMP->mTrackProjX, pMP->mTrackProjY, win, lvl - 1, lvl);
            if (cand.empty()) continue;
            const cv::Mat dMP = pMP->GetDescriptor();
            int d1 = 256, d2 = 256, l1 = -1, l2 = -1, best = -1;
            for (size_t idx : cand) {
                MapPoint* owner = F.mvpMapPoints[idx];
                if (owner && owner->Observations() > 0) continue;
                if (F.mvuRight[idx] > 0 && std::fabs(pMP->mTrackProjXR - F.mvuRight[idx]) > win) continue;
                const int d = Distance(dMP, F.mDescriptors.row((int)idx));
                if (d < d1) {
                    d2 = d1; l2 = l1;
                    d1 = d; l1 = F.mvKeysUn[idx].octave; best = (int)idx;
                } else if (d < d2) {
                    d2 = d; l2 = F.mvKeysUn[idx].octave;
                }
            }
            if (d1 > kHigh) continue;
            if (l1 == l2 && d1 > ratio_ * d2) continue;
            F.mvpMapPoints[(size_t)best] = pMP;
            ++n;
        }
        return n;
    }

    // :1392-1538
    int ProjectLastFrame(Frame& cur, const Frame& last, float th, bool mono) {
        const cv::Mat R = cur.mTcw.rowRange(0, 3).colRange(0, 3);
        const cv::Mat t = cur.mTcw.rowRange(0, 3).col(3);
        const cv::Mat centre = -R.t() * t;   // twc
        const cv::Mat tlc = last.mTcw.rowRange(0, 3).colRange(0, 3) * centre + last.mTcw.rowRange(0, 3).col(3);
        const bool fwd = tlc.at<float>(2) > cur.mb && !mono;
        const bool back = -tlc.at<float>(2) > cur.mb && !mono;
        Histogram hist;
        int n = 0;
        for (int i = 0; i < last.N; ++i) {
            MapPoint* pMP = last.mvpMapPoints[(size_t)i];
            if (!pMP || last.mvbOutlier[(size_t)i]) continue;
            const cv::Mat pc = R * pMP->GetWorldPos() + t;
            const float invz = 1.0 / pc.at<float>(2);
            if (invz < 0) continue;
            const float u = cur.fx * pc.at<float>(0) * invz + cur.cx;
            const float v = cur.fy * pc.at<float>(1) * invz + cur.cy;
            if (u < cur.mnMinX || u > cur.mnMaxX || v < cur.mnMinY || v > cur.mnMaxY) continue;
            const int oct = last.mvKeys[(size_t)i].octave;
            const float rad = th * cur.mvScaleFactors[oct];
            const std::vector<size_t> cand =
                fwd ? cur.GetFeaturesInArea(u, v, rad, oct)
                    : back ? cur.GetFeaturesInArea(u, v, rad, 0, oct)
                           : cur.GetFeaturesInArea(u, v, rad, oct - 1, oct + 1);
            if (cand.empty()) continue;
            const cv::Mat dMP = pMP->GetDescriptor();
            int bd = 256, bi = -1;
            for (size_t i2 : cand) {
                MapPoint* owner = cur.mvpMapPoints[i2];
                if (owner && owner->Observations() > 0) continue;
                if (cur.mvuRight[i2] > 0) {
                    const float ur = u - cur.mbf * invz;
                    if (std::fabs(ur - cur.mvuRight[i2]) > rad) continue;
                }
                const int d = Distance(dMP, cur.mDescriptors.row((int)i2));
                if (d < bd) { bd = d; bi = (int)i2; }
            }
            if (bd > kHigh) continue;
            cur.mvpMapPoints[(size_t)bi] = pMP;
            ++n;
            if (ori_) hist.add(last.mvKeysUn[(size_t)i].angle, cur.mvKeysUn[(size_t)bi].angle, bi);
        }
        if (ori_) n -= hist.filter([&](int idx) { cur.mvpMapPoints[(size_t)idx] = nullptr; });
        return n;
    }

    // :1540-1667
    int ProjectKeyFrame(Frame& cur, KeyFrame* pKF, const std::set<MapPoint*>& found, float th,
                        int orbDist) {
        const cv::Mat R = cur.mTcw.rowRange(0, 3).colRange(0, 3);
        const cv::Mat t = cur.mTcw.rowRange(0, 3).col(3);
        const cv::Mat centre = -R.t() * t;
        const std::vector<MapPoint*> pts = pKF->GetMapPointMatches();
        Histogram hist;
        int n = 0;
        for (size_t i = 0; i < pts.size(); ++i) {
            MapPoint* pMP = pts[i];
            if (!pMP || pMP->isBad() || found.count(pMP)) continue;
            const cv::Mat Xw = pMP->GetWorldPos();
            const cv::Mat pc = R * Xw + t;
            const float invz = 1.0 / pc.at<float>(2);
            const float u = cur.fx * pc.at<float>(0) * invz + cur.cx;
            const float v = cur.fy * pc.at<float>(1) * invz + cur.cy;
            if (u < cur.mnMinX || u > cur.mnMaxX || v < cur.mnMinY || v > cur.mnMaxY) continue;
            const cv::Mat PO = Xw - centre;
            const float dist = cv::norm(PO);
            if (dist < pMP->GetMinDistanceInvariance() || dist > pMP->GetMaxDistanceInvariance()) continue;
            const int lvl = pMP->PredictScale(dist, &cur);
            const std::vector<size_t> cand =
                cur.GetFeaturesInArea(u, v, th * cur.mvScaleFactors[lvl], lvl - 1, lvl + 1);
            if (cand.empty()) continue;
            const cv::Mat dMP = pMP->GetDescriptor();
            int bd = 256, bi = -1;
            for (size_t i2 : cand) {
                if (cur.mvpMapPoints[i2]) continue;
                const int d = Distance(dMP, cur.mDescriptors.row((int)i2));
                if (d < bd) { bd = d; bi = (int)i2; }
            }
            if (bd > orbDist) continue;
            cur.mvpMapPoints[(size_t)bi] = pMP;
            ++n;
            if (ori_) hist.add(pKF->mvKeysUn[i].angle, cur.mvKeysUn[(size_t)bi].angle, bi);
        }
        if (ori_) n -= hist.filter([&](int idx) { cur.mvpMapPoints[(size_t)idx] = nullptr; });
        return n;
    }

    // :321-434
    int ProjectSim3(KeyFrame* pKF, const cv::Mat& Scw, const std::vector<MapPoint*>& pts,
                    std::vector<MapPoint*>& matched, int th) {
        Pose P = decompose(Scw);
        std::set<MapPoint*> found(matched.begin(), matched.end());
        found.erase(nullptr);
        int n = 0;
        for (MapPoint* pMP : pts) {
            if (pMP->isBad() || found.count(pMP)) continue;
            float u, v, ur, dist;
            int lvl;
            if (!view_from(pKF, P, pMP, 1, 0.f, u, v, ur, dist, lvl)) continue;
            const std::vector<size_t> cand = pKF->GetFeaturesInArea(u, v, th * pKF->mvScaleFactors[lvl]);
            if (cand.empty()) continue;
            const cv::Mat dMP = pMP->GetDescriptor();
            int bd = 256, bi = -1;
            for (size_t idx : cand) {
                if (matched[idx]) continue;
                const int o = pKF->mvKeysUn[idx].octave;
                if (o < lvl - 1 || o > lvl) continue;
                const int d = Distance(dMP, pKF->mDescriptors.row((int)idx));
                if (d < bd) { bd = d; bi = (int)idx; }
            }
            if (bd > kLow) continue;
            matched[(size_t)bi] = pMP;
            ++n;
        }
        return n;
    }

    // :182-319
    int BowKeyFrameFrame(KeyFrame* pKF, Frame& F, std::vector<MapPoint*>& out) {
        const std::vector<MapPoint*> kfPts = pKF->GetMapPointMatches();
        out.assign((size_t)F.N, nullptr);
        Histogram hist;
        int n = 0;
        for_shared_nodes(pKF->mFeatVec, F.mFeatVec, [&](const std::vector<unsigned>& a,
                                                        const std::vector<unsigned>& b) {
            for (unsigned ia : a) {
                MapPoint* pMP = kfPts[ia];
                if (!pMP || pMP->isBad()) continue;
                const cv::Mat da = pKF->mDescriptors.row((int)ia);
                int d1 = 256, d2 = 256, best = -1;
                for (unsigned ib : b) {
                    if (out[ib]) continue;
                    const int d = Distance(da, F.mDescriptors.row((int)ib));
                    if (d < d1) { d2 = d1; d1 = d; best = (int)ib; }
                    else if (d < d2) d2 = d;
                }
                if (d1 > kLow || !((float)d1 < ratio_ * (float)d2)) continue;
                out[(size_t)best] = pMP;
                if (ori_) hist.add(pKF->mvKeysUn[ia].angle, F.mvKeys[(size_t)best].angle, best);
                ++n;
            }
        });
        if (ori_) n -= hist.filter([&](int idx) { out[(size_t)idx] = nullptr; });
        return n;
    }

    // :563-696
    int BowKeyFrames(KeyFrame* pKF1, KeyFrame* pKF2, std::vector<MapPoint*>& out) {
        const std::vector<MapPoint*> p1 = pKF1->GetMapPointMatches(), p2 = pKF2->GetMapPointMatches();
        out.assign(p1.size(), nullptr);
        std::vector<bool> taken(p2.size(), false);
        Histogram hist;
        int n = 0;
        for_shared_nodes(pKF1->mFeatVec, pKF2->mFeatVec, [&](const std::vector<unsigned>& a,
                                                             const std::vector<unsigned>& b) {
            for (unsigned i1 : a) {
                if (!p1[i1] || p1[i1]->isBad()) continue;
                const cv::Mat d1m = pKF1->mDescriptors.row((int)i1);
                int d1 = 256, d2 = 256, best = -1;
                for (unsigned i2 : b) {
                    if (taken[i2] || !p2[i2] || p2[i2]->isBad()) continue;
                    const int d = Distance(d1m, pKF2->mDescriptors.row((int)i2));
                    if (d < d1) { d2 = d1; d1 = d; best = (int)i2; }
                    else if (d < d2) d2 = d;
                }
                if (!(d1 < kLow) || !((float)d1 < ratio_ * (float)d2)) continue;
                out[i1] = p2[(size_t)best];
                taken[(size_t)best] = true;
                if (ori_) hist.add(pKF1->mvKeysUn[i1].angle, pKF2->mvKeysUn[(size_t)best].angle, (int)i1);
                ++n;
            }
        });
        if (ori_) n -= hist.filter([&](int i1) { out[(size_t)i1] = nullptr; });
        return n;
    }

    // :446-561
    int Initialization(Frame& F1, Frame& F2, std::vector<cv::Point2f>& prev, std::vector<int>& m12,
                       int window) {
        m12.assign(F1.mvKeysUn.size(), -1);
        std::vector<int> bestOf2(F2.mvKeysUn.size(), INT_MAX), m21(F2.mvKeysUn.size(), -1);
        Histogram hist;
        int n = 0;
        for (size_t i1 = 0; i1 < F1.mvKeysUn.size(); ++i1) {
            const int lvl = F1.mvKeysUn[i1].octave;
            if (lvl > 0) continue;
            const std::vector<size_t> cand = F2.GetFeaturesInArea(prev[i1].x, prev[i1].y, window, lvl, lvl);
            if (cand.empty()) continue;
            const cv::Mat d1m = F1.mDescriptors.row((int)i1);
            int d1 = INT_MAX, d2 = INT_MAX, best = -1;
            for (size_t i2 : cand) {
                const int d = Distance(d1m, F2.mDescriptors.row((int)i2));
                if (bestOf2[i2] <= d) continue;
                if (d < d1) { d2 = d1; d1 = d; best = (int)i2; }
                else if (d < d2) d2 = d;
            }
            if (d1 > kLow || !(d1 < (float)d2 * ratio_)) continue;
            if (m21[(size_t)best] >= 0) {   // the feature changes hands
                m12[(size_t)m21[(size_t)best]] = -1;
                --n;
            }
            m12[i1] = best;
            m21[(size_t)best] = (int)i1;
            bestOf2[(size_t)best] = d1;
            ++n;
            if (ori_) hist.add(F1.mvKeysUn[i1].angle, F2.mvKeysUn[(size_t)best].angle, (int)i1);
        }
        if (ori_)
            n -= hist.filter_count([&](int i1) {
                if (m12[(size_t)i1] < 0) return 0;
                m12[(size_t)i1] = -1;
                return 1;
            });
        for (size_t i1 = 0; i1 < m12.size(); ++i1)
            if (m12[i1] >= 0) prev[i1] = F2.mvKeysUn[(size_t)m12[i1]].pt;
        return n;
    }

    // :702-872 with CheckDistEpipolarLine :147-167
    int Triangulation(KeyFrame* pKF1, KeyFrame* pKF2, const cv::Mat& F12,
                      std::vector<std::pair<size_t, size_t>>& pairs, bool onlyStereo) {
        const cv::Mat C2 = pKF2->GetRotation() * pKF1->GetCameraCenter() + pKF2->GetTranslation();
        const float invz = 1.0f / C2.at<float>(2);
        const float ex = pKF2->fx * C2.at<float>(0) * invz + pKF2->cx;
        const float ey = pKF2->fy * C2.at<float>(1) * invz + pKF2->cy;
        std::vector<int> m12((size_t)pKF1->N, -1);
        Histogram hist;
        int n = 0;
        for_shared_nodes(pKF1->mFeatVec, pKF2->mFeatVec, [&](const std::vector<unsigned>& a,
                                                             const std::vector<unsigned>& b) {
            for (unsigned i1 : a) {
                if (pKF1->GetMapPoint(i1)) continue;
                const bool s1 = pKF1->mvuRight[i1] >= 0;
                if (onlyStereo && !s1) continue;
                const cv::KeyPoint& k1 = pKF1->mvKeysUn[i1];
                const cv::Mat d1m = pKF1->mDescriptors.row((int)i1);
                int bd = kLow, best = -1;
                for (unsigned i2 : b) {
                    if (pKF2->GetMapPoint(i2)) continue;   // vbMatched2 is never set (:722)
                    const bool s2 = pKF2->mvuRight[i2] >= 0;
                    if (onlyStereo && !s2) continue;
                    const int d = Distance(d1m, pKF2->mDescriptors.row((int)i2));
                    if (d > kLow || d > bd) continue;   // ties: the later one wins
                    const cv::KeyPoint& k2 = pKF2->mvKeysUn[i2];
                    if (!s1 && !s2) {
                        const float dx = ex - k2.pt.x, dy = ey - k2.pt.y;
                        if (dx * dx + dy * dy < 100 * pKF2->mvScaleFactors[(size_t)k2.octave]) continue;
                    }
                    if (epipolar_ok(k1, k2, F12, pKF2)) { best = (int)i2; bd = d; }
                }
                if (best < 0) continue;
                m12[i1] = best;
                ++n;
                if (ori_) hist.add(k1.angle, pKF2->mvKeysUn[(size_t)best].angle, (int)i1);
            }
        });
        if (ori_) n -= hist.filter([&](int i1) { m12[(size_t)i1] = -1; });
        pairs.clear();
        for (size_t i = 0; i < m12.size(); ++i)
            if (m12[i] >= 0) pairs.push_back(std::make_pair(i, (size_t)m12[i]));
        return n;
    }

    // :1158-1382
    int Sim3(KeyFrame* pKF1, KeyFrame* pKF2, std::vector<MapPoint*>& m12, float s12,
             const cv::Mat& R12, const cv::Mat& t12, float th) {
        const cv::Mat sR12 = s12 * R12;
        const cv::Mat sR21 = (1.0 / s12) * R12.t();
        const cv::Mat t21 = -sR21 * t12;
        const std::vector<MapPoint*> p1 = pKF1->GetMapPointMatches(), p2 = pKF2->GetMapPointMatches();
        std::vector<bool> done1(p1.size(), false), done2(p2.size(), false);
        for (size_t i = 0; i < p1.size(); ++i) {
            if (!m12[i]) continue;
            done1[i] = true;
            const int j = m12[i]->GetIndexInKeyFrame(pKF2);
            if (j >= 0 && j < (int)p2.size()) done2[(size_t)j] = true;
        }
        // best keypoint of `to` for each point of `pts` (or -1), intrinsics of pKF1 throughout
        auto one_way = [&](const std::vector<MapPoint*>& pts, const std::vector<bool>& done,
                           KeyFrame* from, const cv::Mat& sR, const cv::Mat& t, KeyFrame* to) {
            std::vector<int> res(pts.size(), -1);
            const cv::Mat Rw = from->GetRotation(), tw = from->GetTranslation();
            for (size_t i = 0; i < pts.size(); ++i) {
                MapPoint* pMP = pts[i];
                if (!pMP || done[i] || pMP->isBad()) continue;
                const cv::Mat pc = sR * (Rw * pMP->GetWorldPos() + tw) + t;
                if (pc.at<float>(2) < 0.0) continue;
                const float invz = 1.0 / pc.at<float>(2);
                const float u = pKF1->fx * (pc.at<float>(0) * invz) + pKF1->cx;
                const float v = pKF1->fy * (pc.at<float>(1) * invz) + pKF1->cy;
                if (!to->IsInImage(u, v)) continue;
                const float dist = cv::norm(pc);
                if (dist < pMP->GetMinDistanceInvariance() || dist > pMP->GetMaxDistanceInvariance()) continue;
                const int lvl = pMP->PredictScale(dist, to);
                const std::vector<size_t> cand = to->GetFeaturesInArea(u, v, th * to->mvScaleFactors[lvl]);
                if (cand.empty()) continue;
                const cv::Mat dMP = pMP->GetDescriptor();
                int bd = INT_MAX, bi = -1;
                for (size_t idx : cand) {
                    const int o = to->mvKeysUn[idx].octave;
                    if (o < lvl - 1 || o > lvl) continue;
                    const int d = Distance(dMP, to->mDescriptors.row((int)idx));
                    if (d < bd) { bd = d; bi = (int)idx; }
                }
                if (bd <= kHigh) res[i] = bi;
            }
            return res;
        };
        const std::vector<int> a = one_way(p1, done1, pKF1, sR21, t21, pKF2);
        const std::vector<int> b = one_way(p2, done2, pKF2, sR12, t12, pKF1);
        int found = 0;
        for (size_t i1 = 0; i1 < p1.size(); ++i1) {
            const int i2 = a[i1];
            if (i2 >= 0 && b[(size_t)i2] == (int)i1) {
                m12[i1] = p2[(size_t)i2];
                ++found;
            }
        }
        return found;
    }

    // :879-1029
    int FuseKeyFrame(KeyFrame* pKF, const std::vector<MapPoint*>& pts, float th) {
        Pose P{pKF->GetRotation(), pKF->GetTranslation(), pKF->GetCameraCenter()};
        int n = 0;
        for (MapPoint* pMP : pts) {
            if (!pMP || pMP->isBad() || pMP->IsInKeyFrame(pKF)) continue;
            float u, v, ur, dist;
            int lvl;
            if (!view_from(pKF, P, pMP, 0, pKF->mbf, u, v, ur, dist, lvl)) continue;
            const std::vector<size_t> cand = pKF->GetFeaturesInArea(u, v, th * pKF->mvScaleFactors[lvl]);
            if (cand.empty()) continue;
            const cv::Mat dMP = pMP->GetDescriptor();
            int bd = 256, bi = -1;
            for (size_t idx : cand) {
                const cv::KeyPoint& kp = pKF->mvKeysUn[idx];
                if (kp.octave < lvl - 1 || kp.octave > lvl) continue;
                const float ex = u - kp.pt.x, ey = v - kp.pt.y;
                const float isg = pKF->mvInvLevelSigma2[(size_t)kp.octave];
                if (pKF->mvuRight[idx] >= 0) {
                    const float er = ur - pKF->mvuRight[idx];
                    if ((ex * ex + ey * ey + er * er) * isg > 7.8) continue;
                } else if ((ex * ex + ey * ey) * isg > 5.99) {
                    continue;
                }
                const int d = Distance(dMP, pKF->mDescriptors.row((int)idx));
                if (d < bd) { bd = d; bi = (int)idx; }
            }
            if (bd > kLow) continue;
            MapPoint* there = pKF->GetMapPoint((size_t)bi);
            if (!there) {
                pMP->AddObservation(pKF, (size_t)bi);
                pKF->AddMapPoint(pMP, (size_t)bi);
            } else if (!there->isBad()) {
                if (there->Observations() > pMP->Observations()) pMP->Replace(there);
                else there->Replace(pMP);
            }
            ++n;
        }
        return n;
    }

    // :1033-1156
    int FuseSim3(KeyFrame* pKF, const cv::Mat& Scw, const std::vector<MapPoint*>& pts, float th,
                 std::vector<MapPoint*>& replace) {
        Pose P = decompose(Scw);
        const std::set<MapPoint*> already = pKF->GetMapPoints();
        int n = 0;
        for (size_t k = 0; k < pts.size(); ++k) {
            MapPoint* pMP = pts[k];
            if (pMP->isBad() || already.count(pMP)) continue;
            float u, v, ur, dist;
            int lvl;
            if (!view_from(pKF, P, pMP, 2, 0.f, u, v, ur, dist, lvl)) continue;
            const std::vector<size_t> cand = pKF->GetFeaturesInArea(u, v, th * pKF->mvScaleFactors[lvl]);
            if (cand.empty()) continue;
            const cv::Mat dMP = pMP->GetDescriptor();
            int bd = INT_MAX, bi = -1;
            for (size_t idx : cand) {
                const int o = pKF->mvKeysUn[idx].octave;
                if (o < lvl - 1 || o > lvl) continue;
                const int d = Distance(dMP, pKF->mDescriptors.row((int)idx));
                if (d < bd) { bd = d; bi = (int)idx; }
            }
            if (bd > kLow) continue;
            MapPoint* there = pKF->GetMapPoint((size_t)bi);
            if (!there) {
                pMP->AddObservation(pKF, (size_t)bi);
                pKF->AddMapPoint(pMP, (size_t)bi);
            } else if (!there->isBad()) {
                replace[k] = there;
            }
            ++n;
        }
        return n;
    }

private:
    float ratio_;
    bool ori_;

    struct Pose {
        cv::Mat R, t, centre;
    };
    // Scw = [sR | st]: R = sR / s, t = st / s, centre = -R^T t (:329-334, :1041-1046)
    static Pose decompose(const cv::Mat& Scw) {
        const cv::Mat sR = Scw.rowRange(0, 3).colRange(0, 3);
        const float s = std::sqrt(sR.row(0).dot(sR.row(0)));
        Pose p;
        p.R = sR / s;
        p.t = Scw.rowRange(0, 3).col(3) / s;
        p.centre = -p.R.t() * p.t;
        return p;
    }
    // The shared projection test of the keyframe searches: camera coordinates, positive depth,
    // inside the keyframe image, inside the scale-invariance distances, viewing angle under 60
    // degrees, predicted level.  invz_form 0: 1 / z in float (:913); 1: 1 / z, int numerator
    // (:362); 2: 1.0 / z in double (:1075).
    static bool view_from(KeyFrame* pKF, const Pose& P, MapPoint* pMP, int invz_form, float bf,
                          float& u, float& v, float& ur, float& dist, int& lvl) {
        const cv::Mat Xw = pMP->GetWorldPos();
        const cv::Mat pc = P.R * Xw + P.t;
        if (pc.at<float>(2) < 0.0f) return false;
        const float invz = invz_form == 2 ? (float)(1.0 / pc.at<float>(2)) : 1 / pc.at<float>(2);
        u = pKF->fx * (pc.at<float>(0) * invz) + pKF->cx;
        v = pKF->fy * (pc.at<float>(1) * invz) + pKF->cy;
        if (!pKF->IsInImage(u, v)) return false;
        ur = u - bf * invz;
        const cv::Mat PO = Xw - P.centre;
        dist = cv::norm(PO);
        if (dist < pMP->GetMinDistanceInvariance() || dist > pMP->GetMaxDistanceInvariance()) return false;
        if (PO.dot(pMP->GetNormal()) < 0.5 * dist) return false;
        lvl = pMP->PredictScale(dist, pKF);
        return true;
    }
    static bool epipolar_ok(const cv::KeyPoint& k1, const cv::KeyPoint& k2, const cv::Mat& F,
                            KeyFrame* pKF2) {
        const float a = k1.pt.x * F.at<float>(0, 0) + k1.pt.y * F.at<float>(1, 0) + F.at<float>(2, 0);
        const float b = k1.pt.x * F.at<float>(0, 1) + k1.pt.y * F.at<float>(1, 1) + F.at<float>(2, 1);
        const float c = k1.pt.x * F.at<float>(0, 2) + k1.pt.y * F.at<float>(1, 2) + F.at<float>(2, 2);
        const float num = a * k2.pt.x + b * k2.pt.y + c;
        const float den = a * a + b * b;
        if (den == 0) return false;
        return num * num / den < 3.84 * pKF2->mvLevelSigma2[(size_t)k2.octave];
    }
    // the lock-step walk over two FeatureVectors (std::map, ascending node ids), calling
    // f(features_a, features_b) for every node id both hold
    template <class FV, class Fn>
    static void for_shared_nodes(const FV& A, const FV& B, Fn f) {
        auto ia = A.begin();
        auto ib = B.begin();
        while (ia != A.end() && ib != B.end()) {
            if (ia->first == ib->first) {
                f(ia->second, ib->second);
                ++ia;
                ++ib;
            } else if (ia->first < ib->first) {
                ia = A.lower_bound(ib->first);
            } else {
                ib = B.lower_bound(ia->first);
            }
        }
    }
    // rotation histogram (the rotHist / ComputeThreeMaxima pattern, :194-197, :1669-1710)
    struct Histogram {
        std::vector<int> bins[kBins];
        void add(float a1, float a2, int v) {
            float rot = a1 - a2;
            if (rot < 0.0) rot += 360.0f;
            int b = (int)std::round(rot * (1.0f / kBins));
            if (b == kBins) b = 0;
            bins[b].push_back(v);
        }
        void top3(int& i1, int& i2, int& i3) const {
            int m1 = 0, m2 = 0, m3 = 0;
            i1 = i2 = i3 = -1;
            for (int i = 0; i < kBins; ++i) {
                const int s = (int)bins[i].size();
                if (s > m1) { m3 = m2; m2 = m1; m1 = s; i3 = i2; i2 = i1; i1 = i; }
                else if (s > m2) { m3 = m2; m2 = s; i3 = i2; i2 = i; }
                else if (s > m3) { m3 = s; i3 = i; }
            }
            if (m2 < 0.1f * (float)m1) i2 = i3 = -1;
            else if (m3 < 0.1f * (float)m1) i3 = -1;
        }
        // clear(v) for every entry outside the three largest bins; returns the sum of its results
        template <class Clear>
        int filter_count(Clear clear) const {
            int i1, i2, i3, c = 0;
            top3(i1, i2, i3);
            for (int i = 0; i < kBins; ++i)
                if (i != i1 && i != i2 && i != i3)
                    for (int v : bins[i]) c += clear(v);
            return c;
        }
        template <class Clear>
        int filter(Clear clear) const {
            return filter_count([&](int v) { clear(v); return 1; });
        }
    };
};

}  // namespace orbx_oracle

#endif  // ORBX_ORACLE_MATCHER_OBJECTS_H
