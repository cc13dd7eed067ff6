// render/PathTracer.h — the reference's backend interface, restated with the new GPU_HIP backend.
//
// Same class, signatures and semantics as the reference's libs/render/include/render/PathTracer.h:13-51;
// the only change is BackendType::GPU_HIP, created by create_path_tracer (PathTracer.cpp:9-22).
// An App built against the reference switches backend with one line.
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

namespace render
{
	class Scene;
	class RenderSettings;

	class PathTracer
	{
	public:
		enum class BackendType
		{
			CPU_EMBREE,
			GPU_OPTIX,
			GPU_METAL,
			GPU_HIP  // new: MI355X (gfx950) wavefront integrator over libspt_hip.so
		};

		struct RenderResult
		{
			std::vector<uint32_t> image_buffer;  // RGBA8888, R in the high byte (Color.h:7-10)
			uint32_t width = 0;
			uint32_t height = 0;
		};

	public:
		PathTracer() = default;
		virtual ~PathTracer() = default;

		virtual void render() = 0;

		virtual void set_scene(std::shared_ptr<Scene> scene) = 0;
		virtual void set_settings(std::shared_ptr<RenderSettings> settings) = 0;

		virtual std::shared_ptr<Scene> get_scene() const = 0;
		virtual std::shared_ptr<RenderSettings> get_settings() const = 0;

		virtual BackendType get_backend_type() const = 0;
		virtual std::string get_backend_name() const = 0;

		virtual const RenderResult &get_render_result() = 0;

		static std::unique_ptr<PathTracer> create_path_tracer(BackendType backend);
	};
} // namespace render
