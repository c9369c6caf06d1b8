// face_utils.hpp — forwarding header: the reference's <face_utils.hpp> (include/face_utils.hpp) for a caller of the MI355X engine.
// Declares (globally, as the reference): FaceAnnotation, Vote, loadImage, enlargeFace, loadConfigFile, loadAnnotations, getHeadPoseVotesMT, getFacialFeaturesVotesMT, areaUnderCurve, intersect.
// Everything lives in FaceForest.hpp (the C++ drop-in over the C ABI of ffd.h).
#pragma once

#include "FaceForest.hpp"
