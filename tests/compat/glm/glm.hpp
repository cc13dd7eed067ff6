// COMPILE-CHECK SHIM ONLY (tests/test_cpp_interface.py::test_backend_compiles_against_reference_headers).
// glm is not in this image (the reference's glm submodule is empty, .gitmodules:5-7). This declares just
// enough of glm's vec3/vec4/quat/mat4 surface for `g++ -fsyntax-only` of this repo's backend and an
// App-style hand-off snippet against the reference's own headers (Scene.h, Types.h). Nothing built
// with it is linked, run or used for parity; it has no arithmetic semantics worth relying on.
#pragma once

#include <cmath>

namespace glm
{
	struct vec4;
	struct vec3
	{
		float x, y, z;
		vec3() : x(0), y(0), z(0) {}
		explicit vec3(float s) : x(s), y(s), z(s) {}
		vec3(float a, float b, float c) : x(a), y(b), z(c) {}
		explicit vec3(const vec4 &v);
	};
	struct vec4
	{
		float x, y, z, w;
		vec4() : x(0), y(0), z(0), w(0) {}
		explicit vec4(float s) : x(s), y(s), z(s), w(s) {}
		vec4(float a, float b, float c, float d) : x(a), y(b), z(c), w(d) {}
	};
	inline vec3::vec3(const vec4 &v) : x(v.x), y(v.y), z(v.z) {}
	inline vec3 operator+(const vec3 &a, const vec3 &b) { return vec3(a.x + b.x, a.y + b.y, a.z + b.z); }
	inline vec3 operator*(const vec3 &a, const vec3 &b) { return vec3(a.x * b.x, a.y * b.y, a.z * b.z); }
	inline float length(const vec4 &v) { return std::sqrt(v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w); }
	struct mat4
	{
		vec4 c[4];
		mat4() = default;
		explicit mat4(float s) : c{vec4(s, 0, 0, 0), vec4(0, s, 0, 0), vec4(0, 0, s, 0), vec4(0, 0, 0, s)} {}
		vec4 &operator[](int i) { return c[i]; }
		const vec4 &operator[](int i) const { return c[i]; }
		mat4 &operator*=(const mat4 &) { return *this; }
	};
	struct quat
	{
		float w, x, y, z;
		quat() : w(1), x(0), y(0), z(0) {}
		quat(float w_, float x_, float y_, float z_) : w(w_), x(x_), y(y_), z(z_) {}
	};
	inline quat operator*(const quat &a, const quat &) { return a; }
	inline mat4 translate(const mat4 &m, const vec3 &) { return m; }
	inline mat4 scale(const mat4 &m, const vec3 &) { return m; }
	inline mat4 mat4_cast(const quat &) { return mat4(1.0f); }
	inline quat quat_cast(const mat4 &) { return quat(); }
} // namespace glm
