/*
 * TEST INFRASTRUCTURE ONLY -- layout-exact minimal stand-ins of the third-party types the drop-in
 * adapter (adapter/GICPAlignment.{h,cpp}, adapter/Filter_mi355x.cpp) uses from PCL 1.8, Eigen 3,
 * ROS kinetic and sensor_msgs.  None of them is installed in this image; this header lets the
 * adapter pass a real compiler and run against libmgicp.so (tests/test_adapter_build.py).
 *
 * Layouts kept where the adapter depends on them:
 *  - pcl::PointXYZRGB: 32 bytes, 16-byte aligned, x/y/z at 0/4/8 (PCL_ADD_POINT4D union with
 *    data[4]), the colour union (b, g, r, a bytes / float rgb / uint32 rgba) at 16;
 *  - pcl::PointCloud<T>: points vector, width, height, is_dense, header; Ptr = shared pointer;
 *  - Eigen::Matrix4f: 16 floats, COLUMN-major storage behind data(), operator* and ==.
 * Everything else is the minimum the adapter and the replay driver call.
 */
#pragma once

#include <cmath>
#include <cstdarg>
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

namespace pcl
{
struct alignas(16) PointXYZ
{
    union {
        float data[4];
        struct
        {
            float x, y, z;
        };
    };
    PointXYZ() : data{0.f, 0.f, 0.f, 1.f} {}
};

struct alignas(16) PointXYZRGB
{
    union {
        float data[4];
        struct
        {
            float x, y, z;
        };
    };
    union {
        union {
            struct
            {
                std::uint8_t b, g, r, a;
            };
            float rgb;
        };
        std::uint32_t rgba;
    };
    float pad_[3];
    PointXYZRGB() : data{0.f, 0.f, 0.f, 1.f}, rgba(0xff000000u), pad_{0.f, 0.f, 0.f} {}
};

struct PCLHeader
{
    std::uint32_t seq = 0;
    std::uint64_t stamp = 0;
    std::string frame_id;
};

template <class T>
struct PointCloud
{
    typedef std::shared_ptr<PointCloud<T>> Ptr;
    typedef std::shared_ptr<const PointCloud<T>> ConstPtr;
    PCLHeader header;
    std::vector<T> points;  // alignas(16) T: std::allocator honours it under C++17
    std::uint32_t width = 0;
    std::uint32_t height = 0;
    bool is_dense = true;

    std::size_t size() const { return points.size(); }
    bool empty() const { return points.empty(); }
    void push_back(const T& p)
    {
        points.push_back(p);
        width = static_cast<std::uint32_t>(points.size());
        height = 1;
    }
    T& operator[](std::size_t i) { return points[i]; }
    const T& operator[](std::size_t i) const { return points[i]; }
};

template <class T>
void copyPointCloud(const PointCloud<T>& in, PointCloud<T>& out)
{
    out = in;
}
}  // namespace pcl

namespace Eigen
{
class Matrix4f
{
public:
    Matrix4f() { std::memset(d_, 0, sizeof(d_)); }
    static Matrix4f Identity()
    {
        Matrix4f m;
        for (int i = 0; i < 4; ++i)
            m(i, i) = 1.f;
        return m;
    }
    float& operator()(int r, int c) { return d_[c * 4 + r]; }  // column-major like Eigen
    float operator()(int r, int c) const { return d_[c * 4 + r]; }
    float* data() { return d_; }
    const float* data() const { return d_; }
    Matrix4f operator*(const Matrix4f& b) const
    {
        // Eigen's lazy product of two fixed 4x4: column j = ((a0 b0j + a1 b1j) + a2 b2j) + a3 b3j
        Matrix4f o;
        for (int j = 0; j < 4; ++j)
            for (int i = 0; i < 4; ++i)
            {
                float acc = (*this)(i, 0) * b(0, j);
                acc = acc + (*this)(i, 1) * b(1, j);
                acc = acc + (*this)(i, 2) * b(2, j);
                o(i, j) = acc + (*this)(i, 3) * b(3, j);
            }
        return o;
    }
    bool operator==(const Matrix4f& b) const { return std::memcmp(d_, b.d_, sizeof(d_)) == 0; }

private:
    float d_[16];
};
}  // namespace Eigen

namespace sensor_msgs
{
struct PointField
{
    std::string name;
    std::uint32_t offset = 0;
    std::uint8_t datatype = 0;
    std::uint32_t count = 0;
};
struct PointCloud2
{
    pcl::PCLHeader header;
    std::uint32_t height = 0, width = 0;
    std::vector<PointField> fields;
    bool is_bigendian = false;
    std::uint32_t point_step = 0, row_step = 0;
    std::vector<std::uint8_t> data;
    bool is_dense = true;
};
}  // namespace sensor_msgs

namespace ros
{
struct Duration
{
    double s = 0.0;
    double toSec() const { return s; }
};
struct Time
{
    double s = 0.0;
    static void init() {}
    static Time now();
    Duration operator-(const Time& o) const { return Duration{s - o.s}; }
};
void log(const char* level, const char* fmt, ...);
int error_count();  // ROS_ERROR lines so far (test stand-in only)
}  // namespace ros

#define ROS_INFO(...) ::ros::log("INFO", __VA_ARGS__)
#define ROS_WARN(...) ::ros::log("WARN", __VA_ARGS__)
#define ROS_ERROR(...) ::ros::log("ERROR", __VA_ARGS__)
