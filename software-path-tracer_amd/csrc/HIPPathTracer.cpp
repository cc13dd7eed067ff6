// HIPPathTracer.cpp — the GPU_HIP render::PathTracer backend (host C++ above the C-ABI).
//
// Control flow restates render::CPUPathTracer (reference libs/render/src/engines/pathtracer/backends/
// cpu/CPUPathTracer.cpp): render() :43-85, get_render_result() :87-117, invalidate() :119-161,
// rebuild_scene() :328-404. The pixel loop, trace_ray and the resolve run on the GPU
// (spt_render / spt_resolve_rgba8, or both in one launch: spt_render_resolve_rgba8).
#include "HIPPathTracer.h"

#include <cstring>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "render/Scene.h"
#include "render/Types.h"
#include "spt.h"

namespace render
{
	namespace
	{
		// verify(): always-on check that prints and aborts (render_assert.h:15-25).
		void verify(bool condition, const char *message, const char *func, int line)
		{
			if (!condition)
			{
				std::fprintf(stderr, "VERIFY: %s in %s() at %s:%d\n", message, func, __FILE__, line);
				std::abort();
			}
		}
#define SPT_VERIFY(cond, msg) verify((cond), (msg), __func__, __LINE__)

		void verify_spt(spt_ctx *ctx, int rc, const char *what, const char *func, int line)
		{
			if (rc != SPT_OK)
			{
				std::fprintf(stderr, "VERIFY: %s failed (%d): %s in %s() at %s:%d\n", what, rc,
							 ctx ? spt_last_error(ctx) : "", func, __FILE__, line);
				std::abort();
			}
		}
#define SPT_CALL(ctx, call) verify_spt((ctx), (call), #call, __func__, __LINE__)

		// The reference integrator's fixed parameters (CPUPathTracer.cpp:199, :264).
		constexpr uint32_t kReferenceBounces = 4;
		constexpr uint32_t kReferenceRRDepth = 2;
	} // namespace

	HIPPathTracer::HIPPathTracer(int device_id)
	{
		// CPUPathTracer::CPUPathTracer (:25-35): default settings, then device init
		m_renderSettings = std::make_shared<RenderSettings>();
		const int rc = spt_create(&m_ctx, device_id);
		SPT_VERIFY(rc == SPT_OK && m_ctx != nullptr, "HIP device (gfx950) not available");
	}

	HIPPathTracer::~HIPPathTracer()
	{
		spt_destroy(m_ctx); // (unregisters the result buffer before the vector is freed)
	}

	void HIPPathTracer::render()
	{
		SPT_VERIFY(m_ctx != nullptr, "HIP context not initialized");
		SPT_VERIFY(m_scene != nullptr, "Scene not set before rendering");
		if (m_settingsMode && !m_renderSettings->getProgressive())
			m_frameCount = 0; // a fresh accumulation every call
		invalidate();
		// reference mode: one progressive frame = 1 sample per pixel, seeded with m_frameCount + 1
		// (:61); settings mode: getSamplesPerPixel() such frames in one call (k_paths from 4)
		const uint32_t n = m_settingsMode ? std::max<uint32_t>(1u, m_renderSettings->getSamplesPerPixel()) : 1u;
		m_resolvedAt = 0;
		if (m_outputRegistered && n < SPT_PERSISTENT_MIN_FRAMES)
		{
			// the App reads the result after every render() (App.cpp:230-240): a one-frame call's resolve
			// rides in the frame's own launch, its pixels stored into the registered result buffer as their
			// paths end (longer calls keep render() asynchronous and resolve in get_render_result())
			const float exposure = m_settingsMode ? m_renderSettings->getExposure() : 1.0f;
			SPT_CALL(m_ctx, spt_render_resolve_rgba8(m_ctx, m_frameCount, n, m_frameCount + n, exposure,
													 m_render_result.image_buffer.data()));
			m_resolvedAt = m_frameCount + n;
			m_resolvedExposure = exposure;
		}
		else
		{
			SPT_CALL(m_ctx, spt_render(m_ctx, m_frameCount, n));
		}
		m_frameCount += n;
	}

	void HIPPathTracer::set_settings_mode(bool enabled)
	{
		if (enabled != m_settingsMode)
		{
			m_settingsMode = enabled;
			m_modeChanged = true;
		}
	}

	const PathTracer::RenderResult &HIPPathTracer::get_render_result()
	{
		SPT_VERIFY(m_frameCount > 0, "No frames rendered yet");
		const float exposure = m_settingsMode ? m_renderSettings->getExposure() : 1.0f;
		if (m_resolvedAt == m_frameCount && m_resolvedExposure == exposure)
			return m_render_result; // resolved by render() (spt_render_resolve_rgba8), already in host memory
		// device-side resolve: accum / frameCount, clamp, (uint8)(c * 255), rgba_to_uint32
		if (m_settingsMode)
			SPT_CALL(m_ctx, spt_resolve_rgba8_exposure(m_ctx, m_frameCount, m_renderSettings->getExposure(),
													   m_render_result.image_buffer.data()));
		else
			SPT_CALL(m_ctx, spt_resolve_rgba8(m_ctx, m_frameCount, m_render_result.image_buffer.data()));
		return m_render_result;
	}

	void HIPPathTracer::read_accumulation(std::vector<float> &out)
	{
		out.resize((size_t)m_render_result.width * m_render_result.height * 4);
		if (!out.empty())
			SPT_CALL(m_ctx, spt_read_accum(m_ctx, out.data()));
	}

	void HIPPathTracer::invalidate()
	{
		bool needs_rebuild = false;
		if (m_scene->hasChanges())
		{
			m_frameCount = 0;
			m_outputDirty = true;
			needs_rebuild = true;
		}
		bool reconfigure = false;
		if (m_modeChanged)
		{
			m_frameCount = 0;
			m_outputDirty = true;
			m_modeChanged = false;
			reconfigure = true;
		}
		if (m_renderSettings->isDirty())
		{
			m_frameCount = 0;
			m_outputDirty = true;
			m_renderSettings->clearDirty();
			reconfigure = true;
		}
		if (m_render_result.width != m_renderSettings->getWidth() || m_render_result.height != m_renderSettings->getHeight())
		{
			m_render_result.width = m_renderSettings->getWidth();
			m_render_result.height = m_renderSettings->getHeight();
			// the result buffer is page-locked and GPU-mapped: get_render_result's resolve kernel writes
			// it over PCIe directly (spt_register_host_output); re-registered whenever it reallocates
			SPT_CALL(m_ctx, spt_register_host_output(m_ctx, nullptr, 0));
			m_outputRegistered = false;
			m_render_result.image_buffer.resize((size_t)m_render_result.width * m_render_result.height);
			// (a buffer the runtime cannot register keeps the staging-and-copy resolve: same pixels)
			if (!m_render_result.image_buffer.empty())
				m_outputRegistered = spt_register_host_output(m_ctx, m_render_result.image_buffer.data(),
															  m_render_result.image_buffer.size() * sizeof(uint32_t)) == SPT_OK;
			m_frameCount = 0;
			m_outputDirty = true;
			reconfigure = true;
		}
		if (reconfigure)
		{
			spt_config cfg{};
			cfg.width = m_render_result.width;
			cfg.height = m_render_result.height;
			cfg.max_bounces = m_settingsMode ? m_renderSettings->getMaxBounces() : kReferenceBounces;
			cfg.rr_depth = m_settingsMode ? m_renderSettings->getRussianRouletteDepth() : kReferenceRRDepth;
			cfg.flags = 0;  // ::abs(int) semantics of the reference's Linux build (:320)
			cfg.shard_rank = 0;
			cfg.shard_count = 1;
			cfg.frames_in_flight = 1;  // progressive: one frame per render() call
			SPT_CALL(m_ctx, spt_configure(m_ctx, &cfg));
		}
		if (m_frameCount == 0)
		{
			SPT_CALL(m_ctx, spt_reset(m_ctx));
		}
		if (needs_rebuild)
		{
			rebuild_scene();
			m_scene->markChangesProcessed();
		}
	}

	void HIPPathTracer::rebuild_scene()
	{
		// One sphere primitive per SPHERE_OBJECT node, in registry order (:362-400); one gray
		// Lambertian material (throughput *= 0.7, :260) and the reference sky (:286-292).
		std::vector<spt_prim> prims;
		for (const auto &[id, node] : m_scene->GetAllNodes())
		{
			(void)id;
			if (node->GetType() != NodeType::SPHERE_OBJECT)
				continue;
			const auto *sphere = static_cast<const SphereObject *>(node);
			// glm::vec3 under the reference's Scene.h, render::Vec3 under include/render/Scene.h
			const auto pos = sphere->GetPosition();
			spt_prim p{};
			p.type = SPT_PRIM_SPHERE;
			p.material = 0;
			p.p0[0] = pos.x;
			p.p0[1] = pos.y;
			p.p0[2] = pos.z;
			p.p0[3] = sphere->GetRadius();
			prims.push_back(p);
		}
		spt_material mat{};
		mat.albedo[0] = mat.albedo[1] = mat.albedo[2] = 0.7f;
		spt_env env{};
		env.sky_enabled = 1;
		env.horizon[0] = env.horizon[1] = env.horizon[2] = 1.0f;
		env.zenith[0] = 0.5f;
		env.zenith[1] = 0.7f;
		env.zenith[2] = 1.0f;
		// Same primitive count as the uploaded scene (spheres moved or resized):
		// replace only the changed primitives — a BVH scene is refitted, not rebuilt (spt_update_prims).
		if (m_hasUpload && prims.size() == m_uploaded.size())
		{
			std::vector<uint32_t> idx;
			std::vector<spt_prim> changed;
			for (size_t i = 0; i < prims.size(); ++i)
			{
				if (std::memcmp(&prims[i], &m_uploaded[i], sizeof(spt_prim)) != 0)
				{
					idx.push_back((uint32_t)i);
					changed.push_back(prims[i]);
				}
			}
			SPT_CALL(m_ctx, spt_update_prims(m_ctx, idx.data(), changed.data(), (uint32_t)idx.size()));
		}
		else
		{
			SPT_CALL(m_ctx, spt_set_scene(m_ctx, prims.data(), (uint32_t)prims.size(), &mat, 1, &env));
		}
		m_uploaded = std::move(prims);
		m_hasUpload = true;
	}
} // namespace render
