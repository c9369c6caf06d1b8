// HeadPoseSample.hpp — forwarding header: the reference's <HeadPoseSample.hpp> (include/HeadPoseSample.hpp) for a caller of the MI355X engine.
// Declares (globally, as the reference): HeadPoseSample, HeadPoseLeaf.
// Everything lives in FaceForest.hpp (the C++ drop-in over the C ABI of ffd.h).
#pragma once

#include "FaceForest.hpp"
