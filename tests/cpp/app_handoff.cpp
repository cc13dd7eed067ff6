// Compile-only check (tests/test_cpp_interface.py): the calls the reference App makes on its
// backend — scene building (src/App.cpp:98-133) and the per-frame hand-off (src/App.cpp:230-240) —
// written against render::PathTracer with the GPU_HIP backend selected. Built with -fsyntax-only,
// against the reference's own headers (plus this repo's PathTracer.h, the one-line GPU_HIP enum
// addition) and against this repo's include/render; never linked or run.
#include <cstdint>
#include <cstring>
#include <memory>

#include <glm/glm.hpp>

#include "render/PathTracer.h"
#include "render/Scene.h"
#include "render/Types.h"

void app_like_frame_loop(void *texture_pixels)
{
	auto tracer = render::PathTracer::create_path_tracer(render::PathTracer::BackendType::GPU_HIP);
	auto scene = std::make_shared<render::Scene>();
	{
		auto sphere = scene->CreateNode<render::SphereObject>("123");
		sphere->SetRadius(1.0f);
		sphere->SetPosition(glm::vec3(0.0f, -1.0f, 5.0f));
	}
	for (int x = -5; x <= 5; x += 2)
	{
		auto s = scene->CreateNode<render::SphereObject>("sphere");
		s->SetRadius(0.5f);
		s->SetPosition(glm::vec3((float)x, 1.0f, 10.0f));
	}
	auto settings = std::make_shared<render::RenderSettings>();
	settings->setResolution(512, 512);
	settings->setSamplesPerPixel(64);
	settings->setMaxBounces(8);
	tracer->set_settings(settings);
	tracer->set_scene(scene);

	tracer->render();
	const auto &result = tracer->get_render_result();
	if (result.width > 0 && result.height > 0)
		std::memcpy(texture_pixels, result.image_buffer.data(), (size_t)result.width * result.height * sizeof(uint32_t));
}
