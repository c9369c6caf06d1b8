// Tree.hpp — forwarding header: the reference's <Tree.hpp> (include/Tree.hpp) for a caller of the MI355X engine.
// Declares (globally, as the reference): Tree<S> (the engine's trees; the training constructor grows one on the GPU).
// Everything lives in FaceForest.hpp (the C++ drop-in over the C ABI of ffd.h).
#pragma once

#include "FaceForest.hpp"
