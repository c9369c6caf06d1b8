// MPSample.hpp — forwarding header: the reference's <MPSample.hpp> (include/MPSample.hpp) for a caller of the MI355X engine.
// Declares (globally, as the reference): MPSample (test and training constructors), MPLeaf.
// Everything lives in FaceForest.hpp (the C++ drop-in over the C ABI of ffd.h).
#pragma once

#include "FaceForest.hpp"
