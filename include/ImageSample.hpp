// ImageSample.hpp — forwarding header: the reference's <ImageSample.hpp> (include/ImageSample.hpp) for a caller of the MI355X engine.
// Declares (globally, as the reference): ImageSample (the 38 integral channels, kept on the GPU).
// Everything lives in FaceForest.hpp (the C++ drop-in over the C ABI of ffd.h).
#pragma once

#include "FaceForest.hpp"
