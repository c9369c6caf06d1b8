// Constants.hpp — forwarding header: the reference's <Constants.hpp> (include/Constants.hpp) for a caller of the MI355X engine.
// Declares (globally, as the reference): ForestParam and the class identifiers (TRAIN_IMAGES_PERCENTAGE, NUM_HEADPOSE_CLASSES, ...).
// Everything lives in FaceForest.hpp (the C++ drop-in over the C ABI of ffd.h).
#pragma once

#include "FaceForest.hpp"
