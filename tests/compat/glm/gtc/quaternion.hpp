// COMPILE-CHECK SHIM ONLY: see ../glm.hpp.
#pragma once
#include "../glm.hpp"
