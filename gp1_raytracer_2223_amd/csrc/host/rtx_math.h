// rtx_math.h — host-side value types with the reference's exact IEEE-754 binary32
// operation order (compiled with -ffp-contract=off, never -ffast-math): every result
// here must be bit-identical to the reference's Vector3/Vector4/Matrix
// (source/Vector3.cpp, source/Vector4.cpp, source/Matrix.cpp) because the BVH layout
// and the world-space geometry the GPU sees are derived from them.
#pragma once
#include <cfloat>
#include <cmath>

namespace rtx {

constexpr float kPi = 3.14159265358979323846f;        // MathHelpers.h:7
constexpr float kPi2 = 6.283185307179586476925f;      // MathHelpers.h:10
constexpr float kToRadians = kPi / 180.0f;            // MathHelpers.h:14

// std::min / std::max semantics (b < a ? b : a), which matter for NaN and for the
// FLT_MIN-initialised bounds of the reference BVH builder.
inline float fmin_ref(float a, float b) { return (b < a) ? b : a; }
inline float fmax_ref(float a, float b) { return (a < b) ? b : a; }

struct Vec3 {
    float x{}, y{}, z{};
    Vec3() = default;
    Vec3(float x_, float y_, float z_) : x(x_), y(y_), z(z_) {}

    float SqrMagnitude() const { return x * x + y * y + z * z; }          // Vector3.cpp:27-30
    float Magnitude() const { return sqrtf(x * x + y * y + z * z); }      // :22-25
    float Normalize() {                                                   // :32-40
        const float m = Magnitude();
        x /= m; y /= m; z /= m;
        return m;
    }
    Vec3 Normalized() const { const float m = Magnitude(); return {x / m, y / m, z / m}; }  // :42-46
    float operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }

    Vec3 operator+(const Vec3& v) const { return {x + v.x, y + v.y, z + v.z}; }
    Vec3 operator-(const Vec3& v) const { return {x - v.x, y - v.y, z - v.z}; }
    Vec3 operator*(float s) const { return {x * s, y * s, z * s}; }
    Vec3 operator/(float s) const { return {x / s, y / s, z / s}; }
    Vec3 operator-() const { return {-x, -y, -z}; }

    static float Dot(const Vec3& a, const Vec3& b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
    // Vector3::Cross (:50-54) evaluated literally as UnitX*a - UnitY*b + UnitZ*c.
    static Vec3 Cross(const Vec3& v1, const Vec3& v2) {
        const float a = v1.y * v2.z - v1.z * v2.y;
        const float b = v1.x * v2.z - v1.z * v2.x;
        const float c = v1.x * v2.y - v1.y * v2.x;
        const Vec3 X{1.f * a, 0.f * a, 0.f * a}, Y{0.f * b, 1.f * b, 0.f * b}, Z{0.f * c, 0.f * c, 1.f * c};
        return (X - Y) + Z;
    }
    static Vec3 Min(const Vec3& a, const Vec3& b) { return {fmin_ref(a.x, b.x), fmin_ref(a.y, b.y), fmin_ref(a.z, b.z)}; }
    static Vec3 Max(const Vec3& a, const Vec3& b) { return {fmax_ref(a.x, b.x), fmax_ref(a.y, b.y), fmax_ref(a.z, b.z)}; }
};
inline Vec3 operator*(float s, const Vec3& v) { return {v.x * s, v.y * s, v.z * s}; }

const Vec3 kUnitX{1.f, 0.f, 0.f}, kUnitY{0.f, 1.f, 0.f}, kUnitZ{0.f, 0.f, 1.f};
const Vec3 kMaxVector{FLT_MAX, FLT_MAX, FLT_MAX};
const Vec3 kMinVector{FLT_MIN, FLT_MIN, FLT_MIN};  // Vector3.cpp:14 — FLT_MIN is POSITIVE

struct Vec4 {
    float x{}, y{}, z{}, w{};
    float& at(int i) { return i == 0 ? x : (i == 1 ? y : (i == 2 ? z : w)); }
    float at(int i) const { return i == 0 ? x : (i == 1 ? y : (i == 2 ? z : w)); }
    static float Dot(const Vec4& a, const Vec4& b) { return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w; }  // Vector4.cpp:40-43
};

// Row-major, row-vector convention (source/Matrix.h/.cpp).
struct Mat4 {
    Vec4 d[4]{{1, 0, 0, 0}, {0, 1, 0, 0}, {0, 0, 1, 0}, {0, 0, 0, 1}};
    Mat4() = default;
    Mat4(const Vec3& xa, const Vec3& ya, const Vec3& za, const Vec3& t) {
        d[0] = {xa.x, xa.y, xa.z, 0.f}; d[1] = {ya.x, ya.y, ya.z, 0.f};
        d[2] = {za.x, za.y, za.z, 0.f}; d[3] = {t.x, t.y, t.z, 1.f};
    }
    Vec3 TransformVector(float x, float y, float z) const {                 // Matrix.cpp:35-42
        return {d[0].x * x + d[1].x * y + d[2].x * z, d[0].y * x + d[1].y * y + d[2].y * z,
                d[0].z * x + d[1].z * y + d[2].z * z};
    }
    Vec3 TransformVector(const Vec3& v) const { return TransformVector(v.x, v.y, v.z); }
    Vec3 TransformPoint(float x, float y, float z) const {                  // :49-56
        return {d[0].x * x + d[1].x * y + d[2].x * z + d[3].x, d[0].y * x + d[1].y * y + d[2].y * z + d[3].y,
                d[0].z * x + d[1].z * y + d[2].z * z + d[3].z};
    }
    Vec3 TransformPoint(const Vec3& p) const { return TransformPoint(p.x, p.y, p.z); }
    Mat4 Transposed() const {
        Mat4 r;
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) r.d[i].at(j) = d[j].at(i);
        return r;
    }
    Mat4 operator*(const Mat4& m) const {                                   // :191-205
        Mat4 r;
        const Mat4 mt = m.Transposed();
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) r.d[i].at(j) = Vec4::Dot(d[i], mt.d[j]);
        return r;
    }
    static Mat4 Translation(const Vec3& t) { return Mat4(kUnitX, kUnitY, kUnitZ, t); }
    static Mat4 RotationX(float pitch) {
        const float c = cosf(pitch), s = sinf(pitch);
        return Mat4({1, 0, 0}, {0, c, -s}, {0, s, c}, {0, 0, 0});
    }
    static Mat4 RotationY(float yaw) {                                      // :131-141
        const float c = cosf(yaw), s = sinf(yaw);
        return Mat4({c, 0, -s}, {0, 1, 0}, {s, 0, c}, {0, 0, 0});
    }
    static Mat4 RotationZ(float roll) {
        const float c = cosf(roll), s = sinf(roll);
        return Mat4({c, s, 0}, {-s, c, 0}, {0, 0, 1}, {0, 0, 0});
    }
    static Mat4 Rotation(const Vec3& r) { return RotationX(r.x) * RotationY(r.y) * RotationZ(r.z); }
    static Mat4 Scale(const Vec3& s) { return Mat4({s.x, 0, 0}, {0, s.y, 0}, {0, 0, s.z}, {0, 0, 0}); }
};

struct Color {
    float r{}, g{}, b{};
};

}  // namespace rtx
