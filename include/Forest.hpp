// Forest.hpp — forwarding header: the reference's <Forest.hpp> (include/Forest.hpp) for a caller of the MI355X engine.
// Declares (globally, as the reference): Forest<S> (load, evaluateMT, addTree / getTree / cleanForest).
// Everything lives in FaceForest.hpp (the C++ drop-in over the C ABI of ffd.h).
#pragma once

#include "FaceForest.hpp"
