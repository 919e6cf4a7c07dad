"""Operations console served at ``/`` — the reference website's pages (Website/Packages/datax-pipeline flow designer,
datax-query LiveQuery, datax-jobs, datax-metrics dashboard, datax-home) as one dependency-free page over the REST API:

* Flows: list / create / open;
* Designer tabs: Info, Input (type, mode, connection, schema with *infer from samples*, normalization snippet),
  Reference data, Functions (UDF/UDAF/Azure Function), Query (+ codegen preview + LiveQuery), Rules (tag / alert
  rules with the reference's condition builder — nested and/or groups, field / operator / value, aggregates for
  aggregate rules — turned into SQL by the ``designer/*`` routes, ``dxa.flow.designer``; severity, tag, sinks), Outputs (metric, blob/local, event hub, cosmos db, sql, http,
  file, console), Scale (GPUs), Schedule (batch list) — saved as the Flow JSON the config generator consumes;
* Jobs: state, start / stop / restart;
* Metrics: charts of the flow's metric sources (polling ``/api/metrics/get``, the reference's SumWithTimeChart speed =
  last batch count / polling interval).

Plain HTML + fetch; no build step and no external assets (the deployment has no network).
"""

INDEX_HTML = r"""<!doctype html>
<html><head><meta charset="utf-8"><title>dxa console</title>
<style>
body{font-family:system-ui,sans-serif;margin:0;background:#f4f5f7;color:#222;font-size:14px}
header{background:#1b2a3a;color:#fff;padding:10px 18px;font-size:18px;display:flex;gap:18px;align-items:center}
header a{color:#cfe;cursor:pointer;font-size:14px}
main{padding:14px}
section{background:#fff;border-radius:6px;padding:12px;box-shadow:0 1px 2px #0002;margin-bottom:12px}
table{border-collapse:collapse;width:100%}td,th{border-bottom:1px solid #eee;padding:4px;text-align:left;vertical-align:top}
textarea{width:100%;height:140px;font-family:monospace;font-size:12px}
input,select{margin:2px 4px 2px 0}
.tabs button{margin-right:4px}.tabs .on{background:#1b2a3a;color:#fff}
pre{background:#111;color:#cfc;padding:8px;max-height:260px;overflow:auto;font-size:12px;white-space:pre-wrap}
canvas{width:100%;height:160px;background:#fafafa;border:1px solid #ddd}
.row{display:flex;gap:8px;flex-wrap:wrap;align-items:center}.muted{color:#777}
</style></head><body>
<header>dxa <a onclick="show('flows')">Flows</a><a onclick="show('designer')">Designer</a>
<a onclick="show('jobs')">Jobs</a><a onclick="show('metrics')">Metrics</a><span id="status" class="muted"></span></header>
<main>
<div id="p-flows"><section><h3>Flows</h3><button onclick="newFlow()">New flow</button><table id="flows"></table></section></div>

<div id="p-designer" hidden>
<section><div class="row"><b id="fname">(new flow)</b>
<button onclick="saveFlow()">Save</button><button onclick="flowOp('flow/generateconfigs')">Generate configs</button>
<button onclick="flowOp('flow/startjobs')">Deploy / start</button><button onclick="flowOp('flow/stopjobs')">Stop</button>
<button onclick="flowOp('flow/delete')">Delete</button></div>
<div class="tabs" id="tabs"></div></section>
<section id="tab-info"><h3>Info</h3><div class="row">name <input id="f-name">display name <input id="f-display">
owner <input id="f-owner"></div></section>
<section id="tab-input"><h3>Input</h3><div class="row">type <select id="i-type">
<option>local</option><option>kafka</option><option>events</option><option>iothub</option><option>kafkaeventhub</option>
<option>socket</option><option>file</option><option>blob</option></select>
mode <select id="i-mode"><option>streaming</option><option>batching</option></select>
connection <input id="i-conn" size="40"> topics/hub <input id="i-hub">
batch interval (s) <input id="i-window" size="4" value="1"> max rate <input id="i-rate" size="8" value="1000"></div>
<div class="row">timestamp column <input id="i-ts" value="eventTimeStamp"> watermark <input id="i-wm" size="4" value="0">
<select id="i-wmu"><option>second</option><option>minute</option></select></div>
<p>Schema (Spark StructType JSON) <button onclick="inferSchema()">infer from sample events</button></p>
<textarea id="i-schema"></textarea>
<p>Sample events (JSON lines, for schema inference and LiveQuery)</p><textarea id="i-samples"></textarea>
<p>Normalization snippet (projection)</p><textarea id="i-norm" style="height:60px">Raw.*</textarea></section>
<section id="tab-refdata"><h3>Reference data</h3><table id="refs"></table>
<div class="row">id <input id="r-id"> path <input id="r-path" size="40"> delimiter <input id="r-del" size="2" value=",">
header <select id="r-hdr"><option>true</option><option>false</option></select><button onclick="addRef()">add</button></div></section>
<section id="tab-functions"><h3>Functions</h3><table id="funcs"></table>
<div class="row">id <input id="fn-id"> type <select id="fn-type"><option>jarUDF</option><option>jarUDAF</option>
<option>hipUDF</option><option>hipUDAF</option><option>azureFunction</option></select>
class / endpoint / HIP entry <input id="fn-class" size="30"> return type <input id="fn-rt" size="8" value="double">
argument types <input id="fn-args" size="18" placeholder="double,long"><button onclick="addFunc()">add</button></div>
<p class="muted">hipUDF: a <code>__device__</code> scalar function; hipUDAF: <code>State</code> + init / update / finish
device functions (compiled for the GPU at job start)</p><textarea id="fn-src" style="height:90px"></textarea></section>
<section id="tab-query"><h3>Query</h3>
<textarea id="q-text" style="height:220px">--DataXQuery--
T1 = SELECT * FROM DataXProcessedInput;

OUTPUT T1 TO Metrics;</textarea>
<div class="row"><button onclick="codegen()">Codegen preview</button><button onclick="newKernel()">New LiveQuery kernel</button>
<button onclick="execQuery()">Execute selection / all</button><span id="kernel" class="muted"></span></div></section>
<section id="tab-rules"><h3>Rules</h3><table id="rules"></table>
<div class="row">id <input id="ru-id" size="8"> type <select id="ru-type" onchange="condPreview()"><option>SimpleRule</option>
<option>AggregateRule</option></select> tag <input id="ru-tag" size="8"> severity <select id="ru-sev"><option>Critical</option>
<option>Medium</option><option>Low</option></select> alert <input type="checkbox" id="ru-alert"> sinks <input id="ru-sinks" value="Metrics"></div>
<p>Condition builder (groups of conditions; aggregate rules may aggregate a field)</p><div id="cond"></div>
<div class="row">extra GROUP BY columns <input id="ru-pivots" size="30" placeholder="deviceId,homeId"> condition:
<code id="ru-sql"></code> <span id="ru-err" class="muted"></span><button onclick="addRule()">add rule</button></div></section>
<section id="tab-outputs"><h3>Outputs</h3><table id="outs"></table>
<div class="row">id <input id="o-id" size="10"> type <select id="o-type"><option>metric</option><option>local</option>
<option>blob</option><option>eventhub</option><option>cosmosdb</option><option>sql</option><option>httppost</option>
<option>file</option><option>console</option></select> target <input id="o-target" size="40"
placeholder="folder / connection string / endpoint"><button onclick="addOut()">add</button></div></section>
<section id="tab-scale"><h3>Scale</h3><div class="row">GPUs per job <input id="s-gpus" size="3" value="1"></div></section>
<section id="tab-schedule"><h3>Schedule (batching mode)</h3><table id="sched"></table>
<div class="row">type <select id="b-type"><option>recurring</option><option>oneTime</option></select>
interval <input id="b-int" size="3" value="1"> <select id="b-intt"><option>day</option><option>hour</option>
<option>min</option></select> window <input id="b-win" size="3" value="1"> start <input id="b-start" size="20"
placeholder="2024-01-01T00:00:00Z"> end <input id="b-end" size="20"><button onclick="addBatch()">add</button></div></section>
<section><h3>Result</h3><pre id="out"></pre></section>
</div>

<div id="p-jobs" hidden><section><h3>Jobs</h3><button onclick="refreshJobs()">refresh</button><table id="jobs"></table>
</section></div>

<div id="p-metrics" hidden><section><h3>Metrics</h3><div class="row">flow <select id="m-flow" onchange="loadMetricKeys()">
</select> poll every <input id="m-poll" size="3" value="10">s <button onclick="startPolling()">start</button></div>
<div id="charts"></div></section></div>
</main>
<script>
const TABS=['info','input','refdata','functions','query','rules','outputs','scale','schedule'];
let flow=null, kernelId=null, poll=null;
function $(id){return document.getElementById(id)}
function show(p){for(const x of ['flows','designer','jobs','metrics'])$('p-'+x).hidden=(x!==p);
  if(p==='flows')refreshFlows(); if(p==='jobs')refreshJobs(); if(p==='metrics')loadMetricFlows();}
function tab(t){for(const x of TABS)$('tab-'+x).hidden=(x!==t);
  $('tabs').innerHTML=TABS.map(x=>`<button class="${x===t?'on':''}" onclick="tab('${x}')">${x}</button>`).join('');}
async function api(route, body){const r=await fetch('/api/'+route,{method:'POST',headers:{'Content-Type':'application/json'},
  body:JSON.stringify(body===undefined?{}:body)});const j=await r.json();$('out').textContent=JSON.stringify(j,null,1).slice(0,30000);
  $('status').textContent=j.error?('error: '+j.message):'ok';return j;}
function esc(s){return String(s==null?'':s).replace(/[&<>]/g,c=>({'&':'&amp;','<':'&lt;','>':'&gt;'}[c]))}
async function refreshFlows(){const f=await api('flow/getall/min');
  $('flows').innerHTML='<tr><th>name</th><th>display</th><th>owner</th></tr>'+(f.result||[]).map(x=>
  `<tr><td><a href="#" onclick="openFlow('${esc(x.name)}')">${esc(x.name)}</a></td><td>${esc(x.displayName)}</td><td>${esc(x.owner)}</td></tr>`).join('');}
function blankFlow(){return {name:'',gui:{name:'',displayName:'',owner:'',input:{type:'local',mode:'streaming',properties:{
  inputSchemaFile:'',normalizationSnippet:'Raw.*',windowDuration:'1',maxRate:'1000',timestampColumn:'',watermarkValue:'0',
  watermarkUnit:'second'},referenceData:[]},process:{queries:[''],functions:[],jobconfig:{jobNumGpus:'1'}},
  outputs:[{id:'Metrics',type:'metric',properties:{}}],rules:[],batchList:[]}}}
function newFlow(){flow=blankFlow();fill();show('designer');tab('info');renderCond()}
async function openFlow(n){const r=await api('flow/get',{name:n});flow=r.result;fill();show('designer');tab('info');renderCond()}
function fill(){const g=flow.gui,i=g.input,p=i.properties;$('fname').textContent=flow.name||'(new flow)';
  $('f-name').value=flow.name||'';$('f-display').value=g.displayName||'';$('f-owner').value=g.owner||'';
  $('i-type').value=i.type||'local';$('i-mode').value=i.mode||'streaming';$('i-conn').value=p.inputEventhubConnection||'';
  $('i-hub').value=p.inputEventhubName||'';$('i-window').value=p.windowDuration||'1';$('i-rate').value=p.maxRate||'';
  $('i-ts').value=p.timestampColumn||'';$('i-wm').value=p.watermarkValue||'0';$('i-wmu').value=p.watermarkUnit||'second';
  $('i-schema').value=p.inputSchemaFile||'';$('i-norm').value=p.normalizationSnippet||'Raw.*';
  $('q-text').value=(g.process.queries||[''])[0];$('s-gpus').value=(g.process.jobconfig||{}).jobNumGpus||'1';renderLists();}
function collect(){const g=flow.gui,i=g.input,p=i.properties;flow.name=$('f-name').value;g.name=flow.name;
  g.displayName=$('f-display').value||flow.name;g.owner=$('f-owner').value;i.type=$('i-type').value;i.mode=$('i-mode').value;
  p.inputEventhubConnection=$('i-conn').value;p.inputEventhubName=$('i-hub').value;p.windowDuration=$('i-window').value;
  p.maxRate=$('i-rate').value;p.timestampColumn=$('i-ts').value;p.watermarkValue=$('i-wm').value;p.watermarkUnit=$('i-wmu').value;
  p.inputSchemaFile=$('i-schema').value;p.normalizationSnippet=$('i-norm').value;g.process.queries=[$('q-text').value];
  g.process.jobconfig={...(g.process.jobconfig||{}),jobNumGpus:$('s-gpus').value};return flow;}
function renderLists(){const g=flow.gui;
  $('refs').innerHTML=(g.input.referenceData||[]).map((r,k)=>`<tr><td>${esc(r.id)}</td><td>${esc(r.properties.path)}</td><td><button onclick="del('ref',${k})">x</button></td></tr>`).join('');
  $('funcs').innerHTML=(g.process.functions||[]).map((f,k)=>`<tr><td>${esc(f.id)}</td><td>${esc(f.type)}</td><td>${esc(f.properties.class||f.properties.serviceEndpoint||f.properties.entry)}</td><td><button onclick="del('fn',${k})">x</button></td></tr>`).join('');
  $('rules').innerHTML=(g.rules||[]).map((r,k)=>{const p=r.properties;return `<tr><td>${esc(p._S_ruleId)}</td><td>${esc(p._S_ruleType)}</td><td>${esc(p._S_condition)}</td><td>${esc(p._S_tag)}</td><td>${esc(p._S_severity)}</td><td>${p._S_isAlert?'alert':''}</td><td><button onclick="del('rule',${k})">x</button></td></tr>`}).join('');
  $('outs').innerHTML=(g.outputs||[]).map((o,k)=>`<tr><td>${esc(o.id)}</td><td>${esc(o.type)}</td><td>${esc(JSON.stringify(o.properties))}</td><td><button onclick="del('out',${k})">x</button></td></tr>`).join('');
  $('sched').innerHTML=(g.batchList||[]).map((b,k)=>`<tr><td>${esc(b.type)}</td><td>${esc(JSON.stringify(b.properties))}</td><td>${b.disabled?'disabled':''}</td><td><button onclick="del('batch',${k})">x</button></td></tr>`).join('');}
function del(kind,k){const g=flow.gui;({ref:g.input.referenceData,fn:g.process.functions,rule:g.rules,out:g.outputs,batch:g.batchList})[kind].splice(k,1);renderLists();}
function addRef(){flow.gui.input.referenceData.push({id:$('r-id').value,type:'csv',properties:{path:$('r-path').value,delimiter:$('r-del').value,header:$('r-hdr').value==='true'}});renderLists();}
function addFunc(){const t=$('fn-type').value,v=$('fn-class').value;let p;
  if(t==='azureFunction')p={serviceEndpoint:v,api:'',code:'',methodType:'get',params:[]};
  else if(t==='hipUDF'||t==='hipUDAF')p={source:$('fn-src').value,entry:v||$('fn-id').value,returnType:$('fn-rt').value,
    argTypes:$('fn-args').value.split(',').map(x=>x.trim()).filter(x=>x)};
  else p={class:v,path:'',libs:[]};
  flow.gui.process.functions.push({id:$('fn-id').value,type:t,properties:p});renderLists();}
const OPS=[['equal','='],['notEqual','<>'],['greater','>'],['lessThan','<'],['greaterThanOrEqual','>='],
  ['lessThanOrEqual','<='],['stringEqual','= text'],['stringNotEqual','<> text'],['contains','contains'],
  ['notContains','not contains'],['startsWith','starts with'],['endsWith','ends with']];
const AGGS=['none','MIN','MAX','AVG','SUM','COUNT','DCOUNT'];
function newCond(){return {type:'condition',conjunction:'and',field:'',operator:'equal',value:'',aggregate:'none'}}
let ruleConds={type:'group',conjunction:'and',conditions:[newCond()]};
function sel(opts,v,on){return `<select onchange="${on}">`+opts.map(o=>{const [k,t]=Array.isArray(o)?o:[o,o];
  return `<option value="${k}" ${k===v?'selected':''}>${t}</option>`}).join('')+'</select>'}
function nodeAt(path){let n=ruleConds;for(const i of path)n=n.conditions[i];return n}
function setC(path,k,v){nodeAt(path)[k]=v;condPreview()}
function addC(path,grp){nodeAt(path).conditions.push(grp?{type:'group',conjunction:'and',conditions:[newCond()]}:newCond());renderCond()}
function rmC(path){const p=path.slice(0,-1),i=path[path.length-1];nodeAt(p).conditions.splice(i,1);renderCond()}
function condHtml(g,path){const agg=$('ru-type').value==='AggregateRule';
  let h='<div style="border-left:3px solid #9ab;padding-left:8px;margin:4px 0">';
  g.conditions.forEach((c,i)=>{const p=JSON.stringify(path.concat([i]));
    const conj=i?sel(['and','or'],c.conjunction,`setC(${p},'conjunction',this.value)`):'';
    if(c.type==='group'){h+=`<div>${conj} group <button onclick='rmC(${p})'>x</button>`+condHtml(c,path.concat([i]))+'</div>';return}
    h+=`<div class="row">${conj}`+(agg?sel(AGGS,c.aggregate,`setC(${p},'aggregate',this.value)`):'')+
      `<input size="18" placeholder="field" value="${esc(c.field)}" oninput='setC(${p},"field",this.value)'>`+
      sel(OPS,c.operator,`setC(${p},'operator',this.value)`)+
      `<input size="12" placeholder="value" value="${esc(c.value)}" oninput='setC(${p},"value",this.value)'><button onclick='rmC(${p})'>x</button></div>`});
  const pp=JSON.stringify(path);
  return h+`<button onclick='addC(${pp},false)'>+ condition</button><button onclick='addC(${pp},true)'>+ group</button></div>`}
function renderCond(){$('cond').innerHTML=condHtml(ruleConds,[]);condPreview()}
let condOut={};
async function condPreview(){const r=await fetch('/api/designer/conditions/sql',{method:'POST',headers:{'Content-Type':'application/json'},
  body:JSON.stringify({conditions:ruleConds,ruleType:$('ru-type').value,pivots:$('ru-pivots').value.split(',').map(x=>x.trim()).filter(x=>x)})});
  const j=await r.json();condOut=j.result||{};$('ru-sql').textContent=condOut.condition||'';$('ru-err').textContent=condOut.error||'';}
async function addRule(){await condPreview();if(condOut.error){$('status').textContent='rule: '+condOut.error;return}
  const p={_S_ruleId:$('ru-id').value,_S_ruleType:$('ru-type').value,_S_productId:flow.name,_S_ruleDescription:$('ru-id').value,
  _S_condition:condOut.condition,_S_tagName:'Tag',_S_tag:$('ru-tag').value,_S_severity:$('ru-sev').value,
  _S_isAlert:$('ru-alert').checked,_S_alertSinks:$('ru-sinks').value.split(',').filter(x=>x),_S_aggs:condOut.aggs||[],
  _S_pivots:condOut.pivots||[],schemaTableName:'DataXProcessedInput',conditions:JSON.parse(JSON.stringify(ruleConds))};
  flow.gui.rules.push({id:p._S_ruleId,type:'tag',properties:p});ruleConds={type:'group',conjunction:'and',conditions:[newCond()]};
  renderLists();renderCond();}
function addOut(){const t=$('o-type').value,v=$('o-target').value,p={};
  if(t==='local'||t==='blob'){p.folder=v;p.blobPartitionFormat='yyyy/MM/dd/HH';p.format='json';p.compressionType='none'}
  else if(t==='eventhub'||t==='cosmosdb'||t==='sql'){p.connectionString=v}else if(t==='httppost'){p.endpoint=v}
  else if(t==='file'){p.path=v}flow.gui.outputs.push({id:$('o-id').value,type:t,properties:p});renderLists();}
function addBatch(){flow.gui.batchList=flow.gui.batchList||[];flow.gui.batchList.push({id:String(flow.gui.batchList.length),type:$('b-type').value,disabled:false,
  properties:{interval:$('b-int').value,intervalType:$('b-intt').value,delay:'0',delayType:'min',window:$('b-win').value,
  windowType:$('b-intt').value,startTime:$('b-start').value,endTime:$('b-end').value,lastProcessedTime:''}});renderLists();}
async function saveFlow(){collect();const r=await api('flow/save',flow);if(!r.error)$('fname').textContent=flow.name;}
async function flowOp(op){collect();await api(op,{name:flow.name});}
function samples(){return $('i-samples').value.split('\n').filter(l=>l.trim())}
async function inferSchema(){const r=await api('inputdata/inferschema',{name:$('f-name').value,events:samples()});
  if(!r.error)$('i-schema').value=r.result.Schema;}
async function codegen(){collect();await api('userqueries/codegen',{query:$('q-text').value,
  rules:flow.gui.rules.map(r=>{const o={};for(const [k,v] of Object.entries(r.properties))o[k.startsWith('_S_')?'$'+k.slice(3):k]=v;return o})});}
async function newKernel(){await saveFlow();if(samples().length)await api('inputdata/refreshsample',{name:flow.name,events:samples()});
  const r=await api('kernel',{flowName:flow.name});kernelId=r.result;$('kernel').textContent=kernelId?('kernel '+kernelId.slice(0,8)):'';}
async function execQuery(){if(!kernelId)await newKernel();const ta=$('q-text');
  const sel=ta.value.substring(ta.selectionStart,ta.selectionEnd)||ta.value;await api('kernel/executequery',{kernelId,query:sel});}
async function refreshJobs(){const j=await api('job/getall');$('jobs').innerHTML='<tr><th>job</th><th>state</th><th>gpus</th><th></th></tr>'+
  (j.result||[]).map(x=>`<tr><td>${esc(x.name)}</td><td>${esc(x.state)}</td><td>${esc(x.gpus)}</td><td>
  <button onclick="jobOp('job/start','${esc(x.name)}')">start</button><button onclick="jobOp('job/stop','${esc(x.name)}')">stop</button>
  <button onclick="jobOp('job/restart','${esc(x.name)}')">restart</button></td></tr>`).join('');}
async function jobOp(op,n){await api(op,{name:n});refreshJobs();}
async function loadMetricFlows(){const f=await api('flow/getall/min');$('m-flow').innerHTML=(f.result||[]).map(x=>`<option>${esc(x.name)}</option>`).join('');loadMetricKeys();}
let metricKeys=[];
async function loadMetricKeys(){const n=$('m-flow').value;if(!n)return;const r=await api('flow/get',{name:n});
  const srcs=((r.result||{}).metrics||{}).sources||[];metricKeys=[];for(const s of srcs)for(const m of (s.input||{}).metricKeys||[])metricKeys.push(m.name||m);
  if(!metricKeys.length)metricKeys=['DATAX-'+n+':Input_DataXProcessedInput_Events_Count','DATAX-'+n+':Latency-Process'];
  $('charts').innerHTML=metricKeys.map((k,i)=>`<p>${esc(k)} <span id="v${i}" class="muted"></span></p><canvas id="c${i}" width="900" height="160"></canvas>`).join('');}
async function pollOnce(){const now=Date.now();for(let i=0;i<metricKeys.length;i++){
  const r=await fetch(`/api/metrics/get?m=${encodeURIComponent(metricKeys[i])}&s=${now-3600e3}&e=${now}`);const pts=await r.json();draw(i,pts);}}
function draw(i,pts){const c=$('c'+i);if(!c)return;const g=c.getContext('2d');g.clearRect(0,0,c.width,c.height);if(!pts.length)return;
  const xs=pts.map(p=>p.uts),ys=pts.map(p=>+p.val),x0=Math.min(...xs),x1=Math.max(...xs),y1=Math.max(...ys)||1;
  g.beginPath();pts.forEach((p,k)=>{const x=(p.uts-x0)/((x1-x0)||1)*(c.width-20)+10,y=c.height-10-(+p.val)/y1*(c.height-20);k?g.lineTo(x,y):g.moveTo(x,y)});
  g.strokeStyle='#2a6';g.stroke();g.fillText(y1.toFixed(2),2,10);
  const last=ys[ys.length-1],speed=last/(+$('m-poll').value||10);$('v'+i).textContent=`last ${last} (≈${speed.toFixed(1)}/s)`;}
function startPolling(){if(poll)clearInterval(poll);pollOnce();poll=setInterval(pollOnce,(+$('m-poll').value||10)*1000);}
show('flows');
</script></body></html>
"""
