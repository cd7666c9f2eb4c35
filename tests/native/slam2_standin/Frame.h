// ORB-SLAM2 include/Frame.h stand-in (see slam2_standin.h)
#pragma once
#include "slam2_standin.h"
