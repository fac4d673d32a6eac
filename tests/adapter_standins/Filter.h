/*
 * TEST INFRASTRUCTURE ONLY -- stand-in of the reference's include/Filter.h: the class name, the
 * constructor and the two members adapter/Filter_mi355x.cpp defines, with the reference's
 * signatures (/root/reference/include/Filter.h:43,104,140-143) and its leaf_size_ member (:180).
 */
#pragma once

#include <Utils.h>

class Filter
{
    typedef pcl::PointCloud<pcl::PointXYZRGB> PointCloudRGB;

public:
    explicit Filter(double leaf_size) : leaf_size_(leaf_size) {}
    void downsampleCloud(PointCloudRGB::Ptr cloud, PointCloudRGB::Ptr cloud_downsampled);
    static void removeFromCloud(PointCloudRGB::Ptr input_cloud, PointCloudRGB::Ptr substract_cloud,
                                double threshold, PointCloudRGB::Ptr cloud_filtered);

private:
    double leaf_size_;
};
