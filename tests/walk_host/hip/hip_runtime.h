// Host stand-in for <hip/hip_runtime.h> — TEST INFRASTRUCTURE ONLY (tests/walk_host.cpp).
// Lets the device-side walk (csrc/walk.hpp, csrc/solve.hpp) compile as plain host C++ with g++,
// so its logic can be checked against the CPU oracle without a GPU.
#pragma once
#include <climits>
#include <cmath>
#include <cstdint>
using std::atan2;
using std::hypot;
