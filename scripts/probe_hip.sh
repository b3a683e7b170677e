set -x
env | grep -iE "HIP|ROCR|CUDA|HSA|GPU" | sort
python -c "import torch; print('torch alone', torch.cuda.is_available(), torch.cuda.device_count())"
python -c "
import bayesrrcpp_amd as B; print('brr devices', B.lib().brr_device_count())
import torch; print('torch after brr', torch.cuda.is_available())"
python -c "
import torch; print('torch first', torch.cuda.is_available()); x=torch.zeros(3,device='cuda')
import bayesrrcpp_amd as B; print('brr devices after torch', B.lib().brr_device_count())"
ldd bayesrrcpp_amd/libbrr.so | grep -i hip
python -c "import torch,os; d=os.path.dirname(torch.__file__)+'/lib'; print([f for f in os.listdir(d) if 'hip' in f])"
