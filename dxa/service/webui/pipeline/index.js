// datax-pipeline package entry: the flow list and the flow definition pages.
export { FlowListPanel } from './flowList.js';
export { FlowDefinitionPanel } from './flowDefinition.js';
