// Drop-in replacement for the reference's include/TaskBasedPathTracer.hpp: put
// <repo>/include/dropin and <repo>/include before the reference's include/
// directory and link libspt_hip.so; Renderer.hpp then renders on the MI355X.
#pragma once
#include <Globals.hpp>
#include <spt/RenderSegmentShim.hpp>
