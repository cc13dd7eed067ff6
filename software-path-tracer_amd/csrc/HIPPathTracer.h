// HIPPathTracer.h — render::PathTracer backend over libspt_hip.so (the GPU_HIP backend).
//
// Mirrors render::CPUPathTracer (reference libs/render/src/engines/pathtracer/backends/cpu/
// CPUPathTracer.h:21-75) member for member: the same progressive state (frame count, dirty/resize
// handling, backend-owned RenderResult), with the integrator running on an MI355X through the C-ABI
// (include/spt.h). Errors follow the reference's fail-stop convention: verify() prints and aborts
// (render_assert.h:15-25).
#pragma once

#include <memory>
#include <vector>

#include "render/PathTracer.h"
#include "spt.h"

namespace render
{
	class HIPPathTracer : public PathTracer
	{
	public:
		explicit HIPPathTracer(int device_id = 0);
		~HIPPathTracer() override;

		HIPPathTracer(const HIPPathTracer &) = delete;
		HIPPathTracer &operator=(const HIPPathTracer &) = delete;

		void render() override;

		void set_scene(std::shared_ptr<Scene> scene) override { m_scene = scene; }
		void set_settings(std::shared_ptr<RenderSettings> settings) override { m_renderSettings = settings; }

		std::shared_ptr<Scene> get_scene() const override { return m_scene; }
		std::shared_ptr<RenderSettings> get_settings() const override { return m_renderSettings; }

		std::string get_backend_name() const override { return "GPU Path Tracer (HIP, MI355X gfx950)"; }
		BackendType get_backend_type() const override { return BackendType::GPU_HIP; }

		const PathTracer::RenderResult &get_render_result() override;

		// Not in the reference interface: the float RGBA accumulation (W*H*4), for tests and tools.
		void read_accumulation(std::vector<float> &out);
		uint32_t frame_count() const { return m_frameCount; }

		// Not in the reference interface: honour RenderSettings' max bounces,
		// Russian-roulette depth, samples per pixel per render() call, progressive flag and
		// exposure, which CPUPathTracer ignores (CPUPathTracer.cpp:199, :264, :101-104). Off by
		// default: reference mode renders bit-identically to the reference. Takes effect at the
		// next render() (it re-configures and restarts the accumulation).
		void set_settings_mode(bool enabled);
		bool settings_mode() const { return m_settingsMode; }

	private:
		void invalidate();
		void rebuild_scene();

		spt_ctx *m_ctx = nullptr;
		std::vector<spt_prim> m_uploaded;  // the primitives last uploaded (spt_update_prims diffs against them)
		bool m_hasUpload = false;
		std::shared_ptr<Scene> m_scene;
		std::shared_ptr<RenderSettings> m_renderSettings;
		PathTracer::RenderResult m_render_result;
		uint32_t m_frameCount = 0;
		bool m_outputDirty = true;
		bool m_settingsMode = false;
		bool m_modeChanged = false;
		bool m_outputRegistered = false;  // the result buffer is page-locked and GPU-mapped
		uint32_t m_resolvedAt = 0;         // render() resolved the result for this frame count (0: none)
		float m_resolvedExposure = 1.0f;   // ... with this exposure
	};
} // namespace render
