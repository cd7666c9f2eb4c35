// orb_matcher_oracle.cpp — CPU restatement of src/ORBmatcher.cc (TEST INFRASTRUCTURE ONLY).
#include "orb_oracle.h"
