/*
 * adapter/GICPAlignment.cpp -- the reference's GICPAlignment class over the MI355X engine
 * (replaces /root/reference/src/GICPAlignment.cpp; compiled inside the catkin workspace where
 * PCL / Eigen / ROS exist -- they are absent from this image).
 *
 * Behaviour kept from the reference:
 *  - defaults tf 4e-3, 100 iterations, 0.04 m, ransac 1.0 (src/GICPAlignment.cpp:29-32)
 *  - run = config -> [NaN-normal filtering of both clouds] -> fine alignment -> applyTFtoCloud
 *  - every fineAlignment re-sets both inputs (covariances recomputed, as PCL's setInput* reset)
 *  - iterate re-registers the original source with cached grids/covariances, fine_tf = T*fine_tf
 *  - applyTFtoCloud(cloud) writes aligned_cloud_, not cloud
 *  - transform_exists_ only changes on converged runs; getFineTransform logs when false
 *  - every engine failure (invalid / too small cloud, device or transport error) is logged with
 *    ROS_ERROR and leaves transform_exists_ and fine_tf_ untouched (failure row);
 *    a failed fitness query is logged as a failure, never as a score
 */
#include <GICPAlignment.h>

#include <cmath>

namespace
{
static_assert(sizeof(pcl::PointXYZRGB) == 32, "PointXYZRGB record must be 32 bytes (x,y,z,pad,rgb,pad)");

float* xyzOf(pcl::PointCloud<pcl::PointXYZRGB>& c)
{
    return c.points.empty() ? nullptr : &c.points[0].x;
}

void reportEngineError(const mgicp_ctx* ctx, int rc, const char* what)
{
    ROS_ERROR("%s failed (%d): %s", what, rc, mgicp_last_error(ctx));
}
}  // namespace

GICPAlignment::GICPAlignment(PointCloudRGB::Ptr target_cloud, PointCloudRGB::Ptr source_cloud,
                             bool use_covariances)
  : transform_exists_(false), covariances_(use_covariances), engine_(nullptr),
    ransac_outlier_th_(1.0), fine_tf_(Eigen::Matrix4f::Identity()), max_iter_(100),
    tf_epsilon_(4e-3), max_corresp_distance_(4e-2), target_cloud_(target_cloud),
    source_cloud_(source_cloud), aligned_cloud_(new PointCloudRGB), backup_cloud_(new PointCloudRGB)
{
    mgicp_default_params(&engine_params_);
    int rc = mgicp_create(&engine_, &engine_params_);
    if (rc != MGICP_OK)
    {
        ROS_ERROR("MI355X GICP engine unavailable (%d): no HIP device?", rc);
        engine_ = nullptr;
    }
}

GICPAlignment::~GICPAlignment()
{
    mgicp_destroy(engine_);
}

void GICPAlignment::run()
{
    configParameters();
    if (covariances_)
        applyCovariances();
    fineAlignment();
    applyTFtoCloud(source_cloud_);
}

void GICPAlignment::configParameters()
{
    engine_params_.max_iter = max_iter_;
    engine_params_.max_corr_dist = max_corresp_distance_;
    engine_params_.tf_eps = tf_epsilon_;
    if (engine_)
        mgicp_set_params(engine_, &engine_params_);
}

// The reference computes normals (radius = 2 * (res_target + res_source)), drops points whose
// normal is NaN from `cloud` in place, then builds approximate covariances that
// setInputSource/Target discard again.  Only the filtering has an effect, and it is what is
// kept here: NaN normal <=> fewer than 3 points inside the radius.
void GICPAlignment::getCovariances(PointCloudRGB::Ptr cloud)
{
    if (!engine_ || cloud->points.empty())
        return;
    double res_t = 0.0, res_s = 0.0;
    int rc = mgicp_cloud_resolution(engine_, xyzOf(*target_cloud_), target_cloud_->points.size(),
                                    sizeof(pcl::PointXYZRGB), &res_t);
    if (rc == MGICP_OK)
        rc = mgicp_cloud_resolution(engine_, xyzOf(*source_cloud_), source_cloud_->points.size(),
                                    sizeof(pcl::PointXYZRGB), &res_s);
    if (rc != MGICP_OK)
    {
        // no radius, no filtering: leave the cloud as it is rather than filter with radius 0
        reportEngineError(engine_, rc, "cloud resolution");
        return;
    }
    const double radius = (res_t + res_s) * 2.0;
    ROS_INFO("Computing normals with radius: %f", radius);
    std::vector<unsigned char> keep(cloud->points.size(), 0);
    rc = mgicp_radius_filter(engine_, xyzOf(*cloud), cloud->points.size(), sizeof(pcl::PointXYZRGB), radius, 3,
                             keep.data());
    if (rc != MGICP_OK)
    {
        reportEngineError(engine_, rc, "radius filter");
        return;
    }
    PointCloudRGB kept;
    kept.header = cloud->header;
    kept.points.reserve(cloud->points.size());
    for (size_t i = 0; i < keep.size(); ++i)
        if (keep[i])
            kept.points.push_back(cloud->points[i]);
    kept.width = static_cast<uint32_t>(kept.points.size());
    kept.height = 1;
    kept.is_dense = cloud->is_dense;
    *cloud = kept;
}

void GICPAlignment::applyCovariances()
{
    ROS_INFO("Extract covariances from clouds");
    getCovariances(source_cloud_);
    getCovariances(target_cloud_);
}

// one Registration::align: T = final transformation, output = T * source
bool GICPAlignment::alignOnce(PointCloudRGB::Ptr output, Eigen::Matrix4f& T)
{
    if (!engine_)
        return false;
    mgicp_result res;
    Eigen::Matrix4f out = Eigen::Matrix4f::Identity();
    int rc = mgicp_align(engine_, nullptr, out.data(), &res);  // Eigen storage is column-major
    // MGICP_E_SOLVER: PCL's computeTransformation caught the solver exception, broke out of its loop
    // and still ended with final = previous * guess and transformPointCloud(*input_, output, final):
    // the output cloud is written (iterate() overwrites aligned_cloud_, src/GICPAlignment.cpp:116),
    // hasConverged() == false.  The engine returns that final transform on this path.
    const bool solver_failed = rc == MGICP_E_SOLVER;
    if (rc != MGICP_OK && !solver_failed)
    {
        // no cloud, too few points, device / transport failure: the align did not run (PCL's
        // initCompute rejects these before computeTransformation), output and T untouched
        reportEngineError(engine_, rc, "align");
        return false;
    }
    if (output)
    {
        pcl::copyPointCloud(*source_cloud_, *output);
        const int trc = mgicp_transform_source(engine_, out.data(), xyzOf(*output), sizeof(pcl::PointXYZRGB));
        if (trc != MGICP_OK)
        {
            reportEngineError(engine_, trc, "transform of the aligned output");
            return false;
        }
    }
    T = out;
    return !solver_failed && res.converged != 0;
}

// getFitnessScore for the log line; an engine failure is logged as such, never as a score
void GICPAlignment::logFitness(const Eigen::Matrix4f& T)
{
    double fitness = 0.0;
    const int rc = mgicp_fitness(engine_, T.data(), 0.0, &fitness);
    if (rc != MGICP_OK)
        reportEngineError(engine_, rc, "fitness score");
    else
        ROS_INFO("Converged in %f FitnessScore", fitness);
}

void GICPAlignment::fineAlignment()
{
    ROS_INFO("Perform GICP with %d iterations", engine_params_.max_iter);
    if (!engine_)
    {
        ROS_ERROR("GICP no converge");
        return;
    }
    // PCL's setInputSource / setInputTarget + initCompute: an empty or malformed cloud ends the
    // align with an error and converged_ == false -- transform_exists_ and fine_tf_ stay as they were
    int rc = mgicp_set_source(engine_, xyzOf(*source_cloud_), source_cloud_->points.size(), sizeof(pcl::PointXYZRGB));
    if (rc == MGICP_OK)
        rc = mgicp_set_target(engine_, xyzOf(*target_cloud_), target_cloud_->points.size(), sizeof(pcl::PointXYZRGB));
    if (rc != MGICP_OK)
    {
        reportEngineError(engine_, rc, "GICP inputs");
        ROS_ERROR("GICP no converge");
        return;
    }

    ros::Time begin = ros::Time::now();
    ROS_INFO("This step may take a while ...");
    Eigen::Matrix4f T = Eigen::Matrix4f::Identity();
    const bool converged = alignOnce(PointCloudRGB::Ptr(), T);
    ROS_INFO("GICP time: %lf s", (ros::Time::now() - begin).toSec());

    if (!converged)
    {
        ROS_ERROR("GICP no converge");
        return;
    }
    logFitness(T);
    fine_tf_ = T;
    transform_exists_ = Utils::isValidTransform(fine_tf_);
}

void GICPAlignment::iterateFineAlignment(PointCloudRGB::Ptr cloud)
{
    backUp(cloud);
    ROS_INFO("Computing iteration...");
    Eigen::Matrix4f temp_tf = Eigen::Matrix4f::Identity();
    if (!alignOnce(cloud, temp_tf))
    {
        ROS_ERROR("GICP no converge");
        return;
    }
    fine_tf_ = temp_tf * fine_tf_;
    Utils::printTransform(fine_tf_);
    logFitness(temp_tf);
}

void GICPAlignment::iterate()
{
    iterateFineAlignment(aligned_cloud_);
}

void GICPAlignment::backUp(PointCloudRGB::Ptr cloud)
{
    pcl::copyPointCloud(*cloud, *backup_cloud_);
}

void GICPAlignment::undo()
{
    pcl::copyPointCloud(*backup_cloud_, *aligned_cloud_);
}

void GICPAlignment::applyTFtoCloud(PointCloudRGB::Ptr cloud)
{
    pcl::copyPointCloud(*cloud, *aligned_cloud_);
    if (engine_ && !cloud->points.empty())
    {
        const int rc = mgicp_transform_cloud(engine_, fine_tf_.data(), xyzOf(*cloud), cloud->points.size(),
                                             sizeof(pcl::PointXYZRGB), xyzOf(*aligned_cloud_), sizeof(pcl::PointXYZRGB));
        if (rc != MGICP_OK)
            reportEngineError(engine_, rc, "applyTFtoCloud");
    }
}

Eigen::Matrix4f GICPAlignment::getFineTransform()
{
    if (!transform_exists_)
        ROS_ERROR("No transform yet. Please run algorithm");
    return fine_tf_;
}

void GICPAlignment::getAlignedCloud(PointCloudRGB::Ptr aligned_cloud)
{
    pcl::copyPointCloud(*aligned_cloud_, *aligned_cloud);
}

void GICPAlignment::getAlignedCloudROSMsg(sensor_msgs::PointCloud2& aligned_cloud_msg)
{
    Utils::cloudToROSMsg(aligned_cloud_, aligned_cloud_msg);
}

void GICPAlignment::setSourceCloud(PointCloudRGB::Ptr source_cloud) { source_cloud_ = source_cloud; }
void GICPAlignment::setTargetCloud(PointCloudRGB::Ptr target_cloud) { target_cloud_ = target_cloud; }

void GICPAlignment::setMaxIterations(int iterations)
{
    max_iter_ = iterations;
    configParameters();
}

void GICPAlignment::setTfEpsilon(double tf_epsilon)
{
    tf_epsilon_ = tf_epsilon;
    configParameters();
}

void GICPAlignment::setMaxCorrespondenceDistance(int max_corresp_distance)
{
    max_corresp_distance_ = max_corresp_distance;
    configParameters();
}

void GICPAlignment::setRANSACOutlierTh(int ransac_threshold)
{
    ransac_outlier_th_ = ransac_threshold;
    configParameters();
}
