// PathTracer.cpp — backend factory (reference libs/render/src/engines/pathtracer/PathTracer.cpp:9-22)
// with the GPU_HIP case added. CPU_EMBREE stays the reference's own backend (not part of this build).
#include "render/PathTracer.h"

#include <stdexcept>

#include "HIPPathTracer.h"

namespace render
{
	std::unique_ptr<PathTracer> PathTracer::create_path_tracer(BackendType backend)
	{
		switch (backend)
		{
		case BackendType::GPU_HIP:
			return std::make_unique<render::HIPPathTracer>();
		default:
			throw std::runtime_error("Unknown backend type");
		}
	}
} // namespace render
