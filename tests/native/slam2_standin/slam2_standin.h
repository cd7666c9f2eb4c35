// Stand-ins for ORB-SLAM2's Frame, KeyFrame and MapPoint (include/Frame.h, KeyFrame.h,
// MapPoint.h), reduced to the members and methods ORB_SLAM2::ORBmatcher reads or calls, with the
// reference's names and types, so that integration/ORBmatcher.h (the drop-in) and
// oracle/orb_matcher_objects.h (the CPU restatement it is checked against) compile and run in
// tests/native/matcher_test.cpp exactly as they would inside ORB-SLAM2.  The method bodies restate
// the reference's (file:line below); state changes are appended to a log so that two runs of a
// method on two copies of a scene can be compared event by event.  Test infrastructure only.
#ifndef ORBX_SLAM2_STANDIN_H
#define ORBX_SLAM2_STANDIN_H

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <map>
#include <set>
#include <string>
#include <vector>

#include <opencv2/core/core.hpp>

#define FRAME_GRID_ROWS 48
#define FRAME_GRID_COLS 64

namespace DBoW2 {
// Thirdparty/DBoW2/DBoW2/FeatureVector.h: node id -> feature indices
typedef unsigned int NodeId;
class FeatureVector : public std::map<NodeId, std::vector<unsigned int>> {};
}  // namespace DBoW2

namespace ORB_SLAM2 {

class KeyFrame;
class Frame;

// Every state change of a scene, in order ("op id args").
struct SceneLog {
    std::vector<std::string> events;
    void add(const std::string& e) { events.push_back(e); }
};

struct ById {   // std::map<KeyFrame*, size_t> in a stable order across two scene copies
    bool operator()(const KeyFrame* a, const KeyFrame* b) const;
};

class MapPoint {
public:
    long unsigned int mnId = 0;
    SceneLog* log = nullptr;

    // Tracking variables (MapPoint.h:92-97), written by Frame::isInFrustum
    float mTrackProjX = 0.f, mTrackProjY = 0.f, mTrackProjXR = 0.f;
    bool mbTrackInView = false;
    int mnTrackScaleLevel = 0;
    float mTrackViewCos = 0.f;

    cv::Mat mWorldPos;        // 3x1 CV_32F
    cv::Mat mNormalVector;    // 3x1 CV_32F
    cv::Mat mDescriptor;      // 1x32 CV_8U
    std::map<KeyFrame*, size_t, ById> mObservations;
    int nObs = 0;
    bool mbBad = false;
    MapPoint* mpReplaced = nullptr;
    float mfMinDistance = 0.f, mfMaxDistance = 0.f;

    cv::Mat GetWorldPos() { return mWorldPos.clone(); }
    cv::Mat GetNormal() { return mNormalVector.clone(); }
    cv::Mat GetDescriptor() { return mDescriptor.clone(); }
    int Observations() { return nObs; }
    bool isBad() { return mbBad; }
    MapPoint* GetReplaced() { return mpReplaced; }
    inline void AddObservation(KeyFrame* pKF, size_t idx);   // MapPoint.cc:98-109
    bool IsInKeyFrame(KeyFrame* pKF) { return mObservations.count(pKF) > 0; }
    int GetIndexInKeyFrame(KeyFrame* pKF) {
        auto it = mObservations.find(pKF);
        return it == mObservations.end() ? -1 : (int)it->second;
    }
    inline void Replace(MapPoint* pMP);                       // MapPoint.cc:183-221
    float GetMinDistanceInvariance() { return 0.8f * mfMinDistance; }   // MapPoint.cc:394-398
    float GetMaxDistanceInvariance() { return 1.2f * mfMaxDistance; }   // :400-404
    inline int PredictScale(const float& currentDist, KeyFrame* pKF);   // :406-422
    inline int PredictScale(const float& currentDist, Frame* pF);       // :430-444
};

class KeyFrame {
public:
    long unsigned int mnId = 0;
    SceneLog* log = nullptr;
    float fx = 0, fy = 0, cx = 0, cy = 0, invfx = 0, invfy = 0, mbf = 0, mb = 0, mThDepth = 0;
    int N = 0;
    std::vector<cv::KeyPoint> mvKeysUn;
    std::vector<float> mvuRight;   // negative for monocular points
    cv::Mat mDescriptors;
    DBoW2::FeatureVector mFeatVec;
    int mnScaleLevels = 8;
    float mfScaleFactor = 1.2f, mfLogScaleFactor = 0.f;
    std::vector<float> mvScaleFactors, mvLevelSigma2, mvInvLevelSigma2;
    int mnMinX = 0, mnMinY = 0, mnMaxX = 0, mnMaxY = 0;
    int mnGridCols = FRAME_GRID_COLS, mnGridRows = FRAME_GRID_ROWS;
    float mfGridElementWidthInv = 0.f, mfGridElementHeightInv = 0.f;
    std::vector<std::vector<std::vector<size_t>>> mGrid;
    cv::Mat Tcw, Ow;   // 4x4 / 3x1 CV_32F
    std::vector<MapPoint*> mvpMapPoints;

    cv::Mat GetRotation() { return Tcw.rowRange(0, 3).colRange(0, 3).clone(); }
    cv::Mat GetTranslation() { return Tcw.rowRange(0, 3).col(3).clone(); }
    cv::Mat GetCameraCenter() { return Ow.clone(); }
    void AddMapPoint(MapPoint* pMP, const size_t& idx) {   // KeyFrame.cc:207-211
        mvpMapPoints[idx] = pMP;
        if (log) log->add("kf" + std::to_string(mnId) + ".add " + std::to_string(idx) + " mp" + std::to_string(pMP->mnId));
    }
    void EraseMapPointMatch(const size_t& idx) {           // :213-217
        mvpMapPoints[idx] = nullptr;
        if (log) log->add("kf" + std::to_string(mnId) + ".erase " + std::to_string(idx));
    }
    void ReplaceMapPointMatch(const size_t& idx, MapPoint* pMP) {   // :229-232
        mvpMapPoints[idx] = pMP;
        if (log) log->add("kf" + std::to_string(mnId) + ".replace " + std::to_string(idx) + " mp" + std::to_string(pMP->mnId));
    }
    std::set<MapPoint*> GetMapPoints() {                   // :239-252
        std::set<MapPoint*> s;
        for (MapPoint* p : mvpMapPoints)
            if (p && !p->isBad()) s.insert(p);
        return s;
    }
    std::vector<MapPoint*> GetMapPointMatches() { return mvpMapPoints; }
    MapPoint* GetMapPoint(const size_t& idx) { return mvpMapPoints[idx]; }
    bool IsInImage(const float& x, const float& y) const {   // :624-627
        return x >= mnMinX && x < mnMaxX && y >= mnMinY && y < mnMaxY;
    }
    // KeyFrame.cc:583-620
    std::vector<size_t> GetFeaturesInArea(const float& x, const float& y, const float& r) const {
        std::vector<size_t> out;
        const int x0 = std::max(0, (int)std::floor((x - mnMinX - r) * mfGridElementWidthInv));
        if (x0 >= mnGridCols) return out;
        const int x1 = std::min(mnGridCols - 1, (int)std::ceil((x - mnMinX + r) * mfGridElementWidthInv));
        if (x1 < 0) return out;
        const int y0 = std::max(0, (int)std::floor((y - mnMinY - r) * mfGridElementHeightInv));
        if (y0 >= mnGridRows) return out;
        const int y1 = std::min(mnGridRows - 1, (int)std::ceil((y - mnMinY + r) * mfGridElementHeightInv));
        if (y1 < 0) return out;
        for (int ix = x0; ix <= x1; ix++)
            for (int iy = y0; iy <= y1; iy++)
                for (size_t i : mGrid[ix][iy]) {
                    const cv::KeyPoint& kp = mvKeysUn[i];
                    if (std::fabs(kp.pt.x - x) < r && std::fabs(kp.pt.y - y) < r) out.push_back(i);
                }
        return out;
    }
};

inline bool ById::operator()(const KeyFrame* a, const KeyFrame* b) const { return a->mnId < b->mnId; }

class Frame {
public:
    long unsigned int mnId = 0;
    float fx = 0, fy = 0, cx = 0, cy = 0, invfx = 0, invfy = 0;
    float mbf = 0, mb = 0, mThDepth = 0;
    int N = 0;
    std::vector<cv::KeyPoint> mvKeys, mvKeysUn;
    std::vector<float> mvuRight, mvDepth;
    DBoW2::FeatureVector mFeatVec;
    cv::Mat mDescriptors;
    std::vector<MapPoint*> mvpMapPoints;
    std::vector<bool> mvbOutlier;
    // static members in the reference (Frame.h:159-160, 183-186); instance members here
    float mfGridElementWidthInv = 0.f, mfGridElementHeightInv = 0.f;
    std::vector<std::size_t> mGrid[FRAME_GRID_COLS][FRAME_GRID_ROWS];
    cv::Mat mTcw;
    int mnScaleLevels = 8;
    float mfScaleFactor = 1.2f, mfLogScaleFactor = 0.f;
    std::vector<float> mvScaleFactors, mvInvScaleFactors, mvLevelSigma2, mvInvLevelSigma2;
    float mnMinX = 0, mnMaxX = 0, mnMinY = 0, mnMaxY = 0;
    cv::Mat mRcw, mtcw, mRwc, mOw;

    // Frame::UpdatePoseMatrices (Frame.cc:276-282)
    void UpdatePoseMatrices() {
        mRcw = mTcw.rowRange(0, 3).colRange(0, 3);
        mRwc = mRcw.t();
        mtcw = mTcw.rowRange(0, 3).col(3);
        mOw = -mRcw.t() * mtcw;
    }
    // Frame.cc:285-349
    bool isInFrustum(MapPoint* pMP, float viewingCosLimit) {
        pMP->mbTrackInView = false;
        cv::Mat P = pMP->GetWorldPos();
        const cv::Mat Pc = mRcw * P + mtcw;
        const float PcX = Pc.at<float>(0), PcY = Pc.at<float>(1), PcZ = Pc.at<float>(2);
        if (PcZ < 0.0f) return false;
        const float invz = 1.0f / PcZ;
        const float u = fx * PcX * invz + cx;
        const float v = fy * PcY * invz + cy;
        if (u < mnMinX || u > mnMaxX) return false;
        if (v < mnMinY || v > mnMaxY) return false;
        const float maxDistance = pMP->GetMaxDistanceInvariance();
        const float minDistance = pMP->GetMinDistanceInvariance();
        const cv::Mat PO = P - mOw;
        const float dist = cv::norm(PO);
        if (dist < minDistance || dist > maxDistance) return false;
        cv::Mat Pn = pMP->GetNormal();
        const float viewCos = PO.dot(Pn) / dist;
        if (viewCos < viewingCosLimit) return false;
        const int nPredictedLevel = pMP->PredictScale(dist, this);
        pMP->mbTrackInView = true;
        pMP->mTrackProjX = u;
        pMP->mTrackProjXR = u - mbf * invz;
        pMP->mTrackProjY = v;
        pMP->mnTrackScaleLevel = nPredictedLevel;
        pMP->mTrackViewCos = viewCos;
        return true;
    }
    // Frame.cc:351-405
    std::vector<size_t> GetFeaturesInArea(const float& x, const float& y, const float& r,
                                          const int minLevel = -1, const int maxLevel = -1) const {
        std::vector<size_t> out;
        const int x0 = std::max(0, (int)std::floor((x - mnMinX - r) * mfGridElementWidthInv));
        if (x0 >= FRAME_GRID_COLS) return out;
        const int x1 = std::min((int)FRAME_GRID_COLS - 1, (int)std::ceil((x - mnMinX + r) * mfGridElementWidthInv));
        if (x1 < 0) return out;
        const int y0 = std::max(0, (int)std::floor((y - mnMinY - r) * mfGridElementHeightInv));
        if (y0 >= FRAME_GRID_ROWS) return out;
        const int y1 = std::min((int)FRAME_GRID_ROWS - 1, (int)std::ceil((y - mnMinY + r) * mfGridElementHeightInv));
        if (y1 < 0) return out;
        const bool levels = (minLevel > 0) || (maxLevel >= 0);
        for (int ix = x0; ix <= x1; ix++)
            for (int iy = y0; iy <= y1; iy++)
                for (size_t i : mGrid[ix][iy]) {
                    const cv::KeyPoint& kp = mvKeysUn[i];
                    if (levels && (kp.octave < minLevel || (maxLevel >= 0 && kp.octave > maxLevel))) continue;
                    if (std::fabs(kp.pt.x - x) < r && std::fabs(kp.pt.y - y) < r) out.push_back(i);
                }
        return out;
    }
};

inline void MapPoint::AddObservation(KeyFrame* pKF, size_t idx) {
    if (mObservations.count(pKF)) return;
    mObservations[pKF] = idx;
    nObs += pKF->mvuRight[idx] >= 0 ? 2 : 1;
    if (log) log->add("mp" + std::to_string(mnId) + ".obs kf" + std::to_string(pKF->mnId) + " " + std::to_string(idx));
}

inline void MapPoint::Replace(MapPoint* pMP) {
    if (pMP->mnId == mnId) return;
    std::map<KeyFrame*, size_t, ById> obs = mObservations;
    mObservations.clear();
    mbBad = true;
    mpReplaced = pMP;
    if (log) log->add("mp" + std::to_string(mnId) + ".replaced_by mp" + std::to_string(pMP->mnId));
    for (auto& o : obs) {
        if (!pMP->IsInKeyFrame(o.first)) {
            o.first->ReplaceMapPointMatch(o.second, pMP);
            pMP->AddObservation(o.first, o.second);
        } else {
            o.first->EraseMapPointMatch(o.second);
        }
    }
}

// std::log / std::ceil of floats: logf / ceilf (`using namespace std` reaches MapPoint.cc through
// TemplatedVocabulary.h:36, so the float overloads are the ones called)
inline int MapPoint::PredictScale(const float& currentDist, KeyFrame* pKF) {
    const float ratio = mfMaxDistance / currentDist;
    int nScale = (int)std::ceil(std::log(ratio) / pKF->mfLogScaleFactor);
    if (nScale < 0) nScale = 0;
    else if (nScale >= pKF->mnScaleLevels) nScale = pKF->mnScaleLevels - 1;
    return nScale;
}
inline int MapPoint::PredictScale(const float& currentDist, Frame* pF) {
    const float ratio = mfMaxDistance / currentDist;
    int nScale = (int)std::ceil(std::log(ratio) / pF->mfLogScaleFactor);
    if (nScale < 0) nScale = 0;
    else if (nScale >= pF->mnScaleLevels) nScale = pF->mnScaleLevels - 1;
    return nScale;
}

}  // namespace ORB_SLAM2

#endif  // ORBX_SLAM2_STANDIN_H
