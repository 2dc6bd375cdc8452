from gke_ray_train_amd.train.torch import (TorchConfig, TorchTrainer, backward, enable_reproducibility, get_device,
                                           get_devices, prepare_data_loader, prepare_model)
