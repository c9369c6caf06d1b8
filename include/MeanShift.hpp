// MeanShift.hpp — forwarding header: the reference's <MeanShift.hpp> (include/MeanShift.hpp) for a caller of the MI355X engine.
// Declares (globally, as the reference): MeanShiftOption, MeanShift::shift (on the GPU).
// Everything lives in FaceForest.hpp (the C++ drop-in over the C ABI of ffd.h).
#pragma once

#include "FaceForest.hpp"
