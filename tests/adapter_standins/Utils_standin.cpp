/*
 * TEST INFRASTRUCTURE ONLY -- definitions behind the stand-in Utils.h / standin_deps.h.
 * isValidTransform and computeCloudResolution restate /root/reference/src/Utils.cpp:71-82 and
 * :145-174 (brute-force 2-NN instead of the kd-tree: identical result, small test clouds only).
 */
#include <Utils.h>

#include <chrono>
#include <cstring>
#include <limits>

namespace ros
{
Time Time::now()
{
    using namespace std::chrono;
    return Time{duration<double>(steady_clock::now().time_since_epoch()).count()};
}

static int g_errors = 0;
int error_count() { return g_errors; }

void log(const char* level, const char* fmt, ...)
{
    if (std::strcmp(level, "ERROR") == 0)
        ++g_errors;
    std::fprintf(stderr, "[%s] ", level);
    va_list ap;
    va_start(ap, fmt);
    std::vfprintf(stderr, fmt, ap);
    va_end(ap);
    std::fputc('\n', stderr);
}
}  // namespace ros

bool Utils::isValidCloud(PointCloudRGB::Ptr cloud)
{
    return cloud && !cloud->points.empty();
}

bool Utils::isValidTransform(Eigen::Matrix4f transform)
{
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
            if (std::isnan(transform(i, j)))
                return false;
    return true;
}

void Utils::cloudToROSMsg(PointCloudRGB::Ptr cloud, sensor_msgs::PointCloud2& msg, const std::string& frameid)
{
    msg.header.frame_id = frameid;
    msg.height = 1;
    msg.width = static_cast<std::uint32_t>(cloud->points.size());
    msg.point_step = sizeof(pcl::PointXYZRGB);
    msg.row_step = msg.point_step * msg.width;
    msg.fields = {{"x", 0, 7, 1}, {"y", 4, 7, 1}, {"z", 8, 7, 1}, {"rgb", 16, 7, 1}};
    msg.data.resize(msg.row_step);
    if (!cloud->points.empty())
        std::memcpy(msg.data.data(), cloud->points.data(), msg.row_step);
}

double Utils::computeCloudResolution(PointCloudRGB::Ptr cloud)
{
    const auto& p = cloud->points;
    auto finite = [](const pcl::PointXYZRGB& a) {
        return std::isfinite(a.x) && std::isfinite(a.y) && std::isfinite(a.z);
    };
    double res = 0.0;
    int n_points = 0;
    for (std::size_t i = 0; i < p.size(); ++i)
    {
        if (!std::isfinite(p[i].x))
            continue;
        float best = std::numeric_limits<float>::infinity();
        bool found = false;
        for (std::size_t j = 0; j < p.size(); ++j)
        {
            if (j == i || !finite(p[j]))
                continue;
            const float dx = p[i].x - p[j].x, dy = p[i].y - p[j].y, dz = p[i].z - p[j].z;
            float d2 = dx * dx;
            d2 = d2 + dy * dy;
            d2 = d2 + dz * dz;
            if (d2 < best)
                best = d2;
            found = true;
        }
        if (found)
        {
            res += std::sqrt(best);
            ++n_points;
        }
    }
    return n_points ? res / n_points : 0.0;
}

void Utils::printTransform(const Eigen::Matrix4f& t)
{
    for (int i = 0; i < 4; ++i)
        std::fprintf(stderr, "\t\t\t\t[%.4f, %.4f, %.4f, %.4f]\n", t(i, 0), t(i, 1), t(i, 2), t(i, 3));
}
