/*
 * adapter/Filter_mi355x.cpp -- the two Filter members that sit either side of the GICP path,
 * over the MI355X engine.  Replaces the bodies of
 *     Filter::downsampleCloud   (/root/reference/src/Filter.cpp:91-105, pcl::VoxelGrid)
 *     Filter::removeFromCloud   (/root/reference/src/Filter.cpp:176-189, pcl::SegmentDifferences)
 * Delete those two definitions from src/Filter.cpp and add this file to the library sources
 * (INTEGRATION.md section 2); the other Filter members (crop box, RANSAC floor, outliers) keep
 * their PCL implementations.  Compiled inside the catkin workspace (PCL / ROS are absent from
 * this image).
 */
#include <Filter.h>
#include <Utils.h>

#include <mi355x_gicp.h>

#include <cstddef>
#include <mutex>
#include <vector>

namespace
{
static_assert(sizeof(pcl::PointXYZRGB) == 32, "PointXYZRGB record must be 32 bytes (x,y,z,pad,rgb,pad)");
constexpr int kRgbOffset = offsetof(pcl::PointXYZRGB, rgba);

// one engine context per process for the stateless helpers (mgicp_create resolves every kernel).
// A context holds mutable scratch and one stream and serves one caller at a time
// (include/mi355x_gicp.h "Threading"): every use takes helperMutex(), so concurrent ROS
// callbacks (a multi-threaded spinner) serialise on it instead of racing.
std::mutex& helperMutex()
{
    static std::mutex m;
    return m;
}

mgicp_ctx* helperContext()
{
    static mgicp_ctx* ctx = []() {
        mgicp_ctx* c = nullptr;
        if (mgicp_create(&c, nullptr) != MGICP_OK)
        {
            ROS_ERROR("MI355X engine unavailable: no HIP device?");
            return static_cast<mgicp_ctx*>(nullptr);
        }
        return c;
    }();
    return ctx;
}
}  // namespace

void Filter::downsampleCloud(PointCloudRGB::Ptr cloud, PointCloudRGB::Ptr cloud_downsampled)
{
    ROS_INFO("Downsample cloud with leaf_size : %f", leaf_size_);
    double res = Utils::computeCloudResolution(cloud);
    ROS_INFO("Pointcloud resolution before downsampling: %f", res);

    std::lock_guard<std::mutex> lock(helperMutex());
    mgicp_ctx* ctx = helperContext();
    if (!ctx)
        return;
    // the reference passes the leaf through Eigen::Vector4f: round to float first
    const double l = static_cast<float>(leaf_size_);
    const double leaf[3] = {l, l, l};
    PointCloudRGB out;
    out.points.resize(cloud->points.size());
    size_t n_out = 0;
    const int rc = mgicp_voxel_grid(ctx, cloud->points.empty() ? nullptr : &cloud->points[0].x,
                                    cloud->points.size(), sizeof(pcl::PointXYZRGB), kRgbOffset, leaf, 0,
                                    out.points.empty() ? nullptr : &out.points[0].x, sizeof(pcl::PointXYZRGB),
                                    &n_out);
    if (rc != MGICP_OK)
    {
        ROS_ERROR("voxel grid failed (%d): %s", rc, mgicp_last_error(ctx));
        return;
    }
    out.points.resize(n_out);
    out.header = cloud->header;
    out.width = static_cast<uint32_t>(n_out);
    out.height = 1;
    out.is_dense = true;
    *cloud_downsampled = out;

    res = Utils::computeCloudResolution(cloud_downsampled);
    ROS_INFO("Pointcloud resolution after downsampling: %f", res);
}

void Filter::removeFromCloud(PointCloudRGB::Ptr input_cloud, PointCloudRGB::Ptr substract_cloud, double threshold,
                             PointCloudRGB::Ptr cloud_filtered)
{
    ROS_INFO("Difference from segment with threshold: %f", threshold);
    std::lock_guard<std::mutex> lock(helperMutex());
    mgicp_ctx* ctx = helperContext();
    if (!ctx)
        return;
    const size_t n = input_cloud->points.size();
    std::vector<unsigned char> keep(n, 0);
    size_t n_keep = 0;
    const int rc = mgicp_segment_differences(
        ctx, nullptr, n ? &input_cloud->points[0].x : nullptr, n, sizeof(pcl::PointXYZRGB),
        substract_cloud->points.empty() ? nullptr : &substract_cloud->points[0].x, substract_cloud->points.size(),
        sizeof(pcl::PointXYZRGB), threshold, keep.data(), &n_keep);
    if (rc != MGICP_OK)
    {
        ROS_ERROR("segment differences failed (%d): %s", rc, mgicp_last_error(ctx));
        return;
    }
    PointCloudRGB out;
    out.header = input_cloud->header;
    out.points.reserve(n_keep);
    for (size_t i = 0; i < n; ++i)
        if (keep[i])
            out.points.push_back(input_cloud->points[i]);
    out.width = static_cast<uint32_t>(out.points.size());
    out.height = 1;
    out.is_dense = true;
    *cloud_filtered = out;
}
